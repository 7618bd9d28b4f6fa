// Compile-time (obs, action, objective) dims of the supported SynthMO envs.
#pragma once
#include <type_traits>

#include "pgm_common.hpp"

namespace pgm {

template <int V>
using ic = std::integral_constant<int, V>;

// (O, A, K): Walker2d/HalfCheetah, Hopper-v2, Hopper-v3, Humanoid, Ant, Swimmer (SURVEY.md §8 header table).
// f(ic<O>, ic<A>, ic<K>) -> int status.
template <class F>
int dispatch_dims(int O, int A, int K, const char* what, F&& f) {
    if (O == 17 && A == 6 && K == 2) return f(ic<17>{}, ic<6>{}, ic<2>{});
    if (O == 11 && A == 3 && K == 2) return f(ic<11>{}, ic<3>{}, ic<2>{});
    if (O == 11 && A == 3 && K == 3) return f(ic<11>{}, ic<3>{}, ic<3>{});
    if (O == 376 && A == 17 && K == 2) return f(ic<376>{}, ic<17>{}, ic<2>{});
    if (O == 27 && A == 8 && K == 2) return f(ic<27>{}, ic<8>{}, ic<2>{});
    if (O == 8 && A == 2 && K == 2) return f(ic<8>{}, ic<2>{}, ic<2>{});
    set_error("%s: unsupported dims O=%d A=%d K=%d (supported: 17/6/2, 11/3/2, 11/3/3, 376/17/2, 27/8/2, 8/2/2)",
              what, O, A, K);
    return PGM_E_UNSUPPORTED;
}

inline int check_dims(const pgm_dims* d, const char* what) {
    if (!d) {
        set_error("%s: null dims", what);
        return PGM_E_INVALID_ARG;
    }
    if (d->P <= 0 || d->N <= 0 || d->T < 0 || d->O <= 0 || d->A <= 0 || d->K <= 0) {
        set_error("%s: non-positive dims P=%d N=%d T=%d O=%d A=%d K=%d", what, d->P, d->N, d->T, d->O, d->A, d->K);
        return PGM_E_SHAPE;
    }
    if (d->H != H) {
        set_error("%s: hidden size %d unsupported (this build is H=%d, model.py:202)", what, d->H, H);
        return PGM_E_UNSUPPORTED;
    }
    if (d->N > 8) {
        set_error("%s: N=%d envs per task > 8 unsupported", what, d->N);
        return PGM_E_UNSUPPORTED;
    }
    return PGM_OK;
}

}  // namespace pgm
