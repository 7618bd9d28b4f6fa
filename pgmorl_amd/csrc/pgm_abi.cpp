// Host plumbing of the C ABI: version, thread-local error string, parameter layout.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>

#include "pgm_common.hpp"

namespace pgm {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int hip_fail(hipError_t e, const char* what) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return PGM_E_HIP;
}

int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, what);
    return PGM_OK;
}

// CUs of the current device, cached per device (the library's only cache: an immutable device property, written with
// the same value by any thread that races on it)
int device_cu_count() {
    static std::atomic<int> cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    if (dev >= 0 && dev < 64) {
        if (const int c = cus[dev].load(std::memory_order_relaxed)) return c;
    }
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) return 1;
    if (dev >= 0 && dev < 64) cus[dev].store(c, std::memory_order_relaxed);
    return c;
}

int check_coresident(const void* kern, int block, size_t smem, int grid, const char* what) {
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, smem);
    if (e != hipSuccess) return hip_fail(e, what);
    int cus = device_cu_count();
#ifdef PGM_TEST_HOOKS
    if (const char* o = getenv("PGM_TEST_RESIDENT_CUS")) cus = atoi(o);  // test build only: pretend a smaller device
#endif
    if (per_cu < 1 || (long long)grid > (long long)per_cu * cus) {
        set_error("%s: %d workgroups of %d threads (%zu B LDS) cannot all be co-resident: occupancy %d per CU x %d "
                  "CUs; shard the tasks over more GPUs", what, grid, block, smem, per_cu, cus);
        return PGM_E_UNSUPPORTED;
    }
    return PGM_OK;
}

DbgDelay dbg_delay_hook() {
    DbgDelay d{0, 0, 0, 0u};
#ifdef PGM_TEST_HOOKS
    const char* s = getenv("PGM_TEST_DELAY");
    if (s && *s) {
        int st = 0, bl = 0, wh = 0;
        unsigned cy = 0;
        if (sscanf(s, "%d:%d:%d:%u", &st, &bl, &wh, &cy) == 4) d = DbgDelay{st, bl, wh, cy};
    }
#endif
    return d;
}

int read_opts(const pgm_launch_opts* o, pgm_launch_opts* out, const char* what) {
    *out = o ? *o : pgm_launch_opts{};
    if (out->update_kernel < PGM_UPDATE_AUTO || out->update_kernel > PGM_UPDATE_VALU ||
        out->update_split < PGM_SPLIT_AUTO || out->update_split > PGM_SPLIT_QUARTERS ||
        (unsigned)out->fs_one_per_cu > 1u || (unsigned)out->rollout_kernel > 1u || (unsigned)out->eval_kernel > 1u) {
        set_error("%s: invalid pgm_launch_opts {%d, %d, %d, %d, %d}", what, out->update_kernel, out->update_split,
                  out->fs_one_per_cu, out->rollout_kernel, out->eval_kernel);
        return PGM_E_INVALID_ARG;
    }
    return PGM_OK;
}

static inline int32_t round_up(int32_t x, int32_t m) { return (x + m - 1) / m * m; }

Layout make_layout(int O, int A, int K, int Hd) {
    const int32_t sizes[PGM_NUM_PARAM_TENSORS] = {
        O * Hd, Hd, Hd * Hd, Hd,   // actor tower
        O * Hd, Hd, Hd * Hd, Hd,   // critic tower
        Hd * K, K,                 // critic_linear
        Hd * A, A,                 // fc_mean
        A};                        // logstd
    Layout L;
    int32_t p = 0;
    for (int i = 0; i < PGM_NUM_PARAM_TENSORS; ++i) {
        L.off[i] = p;
        p = round_up(p + sizes[i], 4);  // 16-byte aligned tensors
    }
    L.total = round_up(p, 64);
    return L;
}

}  // namespace pgm

extern "C" {

int pgm_abi_version(void) { return PGM_ABI_VERSION; }

const char* pgm_last_error(void) { return pgm::g_err; }

int pgm_param_layout(int32_t O, int32_t A, int32_t K, int32_t H, int32_t* offsets, int32_t* total) {
    if (O <= 0 || A <= 0 || K <= 0 || H <= 0 || !offsets || !total) {
        pgm::set_error("pgm_param_layout: bad arguments");
        return PGM_E_INVALID_ARG;
    }
    pgm::Layout L = pgm::make_layout(O, A, K, H);
    for (int i = 0; i < PGM_NUM_PARAM_TENSORS; ++i) offsets[i] = L.off[i];
    *total = L.total;
    return PGM_OK;
}

}  // extern "C"

