/* pgm_host.h -- native (C++, host CPU) generation-boundary path of PG-MORL: the prediction-guided selection's
 * hyperbolic fits, its greedy hypervolume / sparsity knapsack, and the Pareto-archive primitives the boundary
 * calls once per generation.  libpgm_host.so, built with g++ (no GPU runtime).
 *
 * Every entry returns 0 on success or a negative PGM_E_* code (pgm_abi.h values) with a thread-local message in
 * pgm_host_last_error().  Buffers are caller-owned, row-major fp64; nothing is retained between calls.
 * nthreads <= 0 means "as many as the host offers, at most 16".
 */
#ifndef PGM_HOST_H
#define PGM_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGM_HOST_ABI_VERSION 1

int pgm_host_abi_version(void);
const char* pgm_host_last_error(void);

/* predict_hyperbolic's per-objective fit (morl/population_2d.py:86-113, morl/population_3d.py:81-104):
 *   scipy.optimize.least_squares(fun, ones(4), loss='soft_l1', f_scale=20, jac=jac,
 *                                bounds=([0, 0.1, -5, -500], [a_hi, 20, 5, 500]))
 * with fun = (A (e^{a(x-b)} - 1) / (e^{a(x-b)} + 1) + c - y) * w, method 'trf' with the exact (SVD)
 * trust-region solver, ftol = xtol = gtol = 1e-8, max_nfev = 400 (scipy/optimize/_lsq/trf.py trf_bounds,
 * restated).  nfit independent problems; problem i owns rows [off[i], off[i+1]) of x, y, w.
 * params: [nfit][4] = (A, a, b, c); nfev (optional, may be NULL): residual evaluations per problem. */
int pgm_fit_hyperbolic(int64_t nfit, const int64_t* off, const double* x, const double* y, const double* w,
                       const double* a_hi, double* params, int32_t* nfev, int nthreads);

/* get_ep_indices' membership (morl/utils.py:24-39): keep[i] = 1 iff objs[i] >= 0 in every objective and no
 * point j satisfies objs[j] >= objs[i] everywhere and > somewhere.  objs: [n][k].  (The obj0 ordering stays with
 * the caller's np.argsort, whose tie order is numpy's.) */
int pgm_ep_mask(int64_t n, int k, const double* objs, uint8_t* keep);

/* compute_hypervolume (morl/utils.py:80-84 -> morl/hypervolume.py:41-74): volume dominated by the points with
 * every coordinate >= 0, reference point the origin, rounded to 4 decimals.  k in {1, 2, 3}. */
int pgm_hypervolume(int64_t n, int k, const double* objs, double* hv);

/* The greedy knapsack of prediction_guided_selection: n_pick rounds; each scores every unpicked candidate c by
 * HV(E_c) - alpha * sparsity(E_c), E_c = the virtual EP with prediction c inserted, takes the first maximum
 * (strict >, index order), and inserts it into the virtual EP (the new virtual EP = E_c).
 *   mode PGM_SELECT_STAIRCASE (k = 2, morl/population_2d.py:185-202,262-304): E_c = the EP indices of
 *     (virtual EP + [c]); staircase HV; sparsity = mean squared step between consecutive points in obj0 order;
 *   mode PGM_SELECT_UPDATE_EP (k = 2 or 3, morl/population_3d.py:190-237,296-333): E_c = update_ep(virtual EP, c)
 *     (morl/utils.py:41-66); compute_hypervolume as above; utils.compute_sparsity.
 * ep: [n_ep][k] (the EP's objectives, in the EP's order); preds: [n_cand][k].  picks[n_pick] receives the
 * candidate indices; *n_picked how many rounds found a candidate (fewer when they run out: "Too few
 * candidates"). */
#define PGM_SELECT_STAIRCASE 0
#define PGM_SELECT_UPDATE_EP 1
int pgm_select_greedy(int k, int mode, int64_t n_ep, const double* ep, int64_t n_cand, const double* preds, double alpha,
                      int n_pick, int nthreads, int32_t* picks, int32_t* n_picked);

#ifdef __cplusplus
}
#endif

#endif /* PGM_HOST_H */
