// Native generation-boundary path (host CPU, g++): the prediction-guided selection's hyperbolic fits and greedy
// knapsack, and the Pareto-archive primitives (include/pgm_host.h).  SURVEY.md §8(f) ranks 2-3: these ran as
// Python / scipy once per generation and were the whole run's Amdahl term (55% of a Walker pop = 40 run).
//
// Reference semantics (paths relative to the reference tree):
//   hyperbolic model + soft-L1 least_squares      morl/population_2d.py:86-113, morl/population_3d.py:81-104
//   scipy least_squares 'trf' (bounded, exact)    scipy/optimize/_lsq/trf.py trf_bounds + _lsq/common.py
//                                                 (third-party: restated from its published algorithm)
//   get_ep_indices                                morl/utils.py:24-39
//   update_ep                                     morl/utils.py:41-66
//   compute_hypervolume / compute_sparsity        morl/utils.py:80-100, morl/hypervolume.py:41-74
//   2-D staircase HV / EP-order sparsity          morl/population_2d.py:185-202
//   greedy knapsack                               morl/population_2d.py:262-304, morl/population_3d.py:296-333
#include "pgm_host.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

namespace {

constexpr int E_INVALID_ARG = -1;
constexpr double EPS = 2.220446049250313e-16;  // np.finfo(float).eps
constexpr double INF = std::numeric_limits<double>::infinity();

thread_local char g_err[256];
int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int resolve_threads(int nthreads, int64_t work) {
    int n = nthreads > 0 ? nthreads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    return (int)std::max<int64_t>(1, std::min<int64_t>(n, work));
}

// fn(i) for i in [0, n) over nt threads (dynamic: one atomic counter)
template <class Fn>
void parallel_for(int64_t n, int nt, Fn fn) {
    if (nt <= 1 || n <= 1) {
        for (int64_t i = 0; i < n; ++i) fn(i);
        return;
    }
    std::atomic<int64_t> next{0};
    auto body = [&]() {
        for (int64_t i; (i = next.fetch_add(1)) < n;) fn(i);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(body);
    body();
    for (auto& t : th) t.join();
}

// ===================================================================================== trust-region least squares
constexpr int NP = 4;  // (A, a, b, c)
constexpr double F_SCALE = 20.0, FTOL = 1e-8, XTOL = 1e-8, GTOL = 1e-8;
constexpr int MAX_NFEV = 100 * NP;  // least_squares: max_nfev = 100 n for 'trf'

double norm4(const double* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]); }
double dot4(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3]; }

struct Problem {
    int m;
    const double *x, *y, *w;
    double lb[NP], ub[NP];

    // residuals of the weighted hyperbolic model (population_2d.py:86-88)
    void fun(const double* p, double* f) const {
        for (int i = 0; i < m; ++i) {
            const double e = std::exp(p[1] * (x[i] - p[2]));
            f[i] = (p[0] * (e - 1.) / (e + 1.) + p[3] - y[i]) * w[i];
        }
    }
    // Jacobian [m][4] (population_2d.py:90-108)
    void jac(const double* p, double* J) const {
        const double A = p[0], a = p[1], b = p[2];
        for (int i = 0; i < m; ++i) {
            const double e = std::exp(a * (x[i] - b));
            const double ep1 = e + 1.;
            J[4 * i + 0] = ((e - 1.) / ep1) * w[i];
            J[4 * i + 1] = (A * (x[i] - b) * (2. * e) / (ep1 * ep1)) * w[i];
            J[4 * i + 2] = (A * (-a) * (2. * e) / (ep1 * ep1)) * w[i];
            J[4 * i + 3] = w[i];
        }
    }
};

// soft_l1 with f_scale (least_squares.py construct_loss_function / soft_l1)
double cost_only(const double* f, int m) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) {
        const double z = (f[i] / F_SCALE) * (f[i] / F_SCALE);
        s += 2.0 * (std::sqrt(1.0 + z) - 1.0);
    }
    return 0.5 * F_SCALE * F_SCALE * s;
}
// rho, cost, then scale_for_robust_loss_function on (J, f) in place; returns the cost
double robust_scale(double* J, double* f, int m) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) {
        const double z = (f[i] / F_SCALE) * (f[i] / F_SCALE);
        const double t = 1.0 + z;
        const double r0 = 2.0 * (std::sqrt(t) - 1.0) * (F_SCALE * F_SCALE);
        const double r1 = 1.0 / std::sqrt(t);
        const double r2 = -0.5 * std::pow(t, -1.5) / (F_SCALE * F_SCALE);
        s += r0;
        double js = r1 + 2.0 * r2 * f[i] * f[i];
        if (js < EPS) js = EPS;
        js = std::sqrt(js);
        f[i] *= r1 / js;
        for (int j = 0; j < NP; ++j) J[4 * i + j] *= js;
    }
    return 0.5 * s;
}

void grad(const double* J, const double* f, int m, double* g) {
    for (int j = 0; j < NP; ++j) g[j] = 0.0;
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < NP; ++j) g[j] += J[4 * i + j] * f[i];
}

// common.py CL_scaling_vector
void cl_scaling(const double* x, const double* g, const double* lb, const double* ub, double* v, double* dv) {
    for (int j = 0; j < NP; ++j) {
        v[j] = 1.0;
        dv[j] = 0.0;
        if (g[j] < 0 && std::isfinite(ub[j])) {
            v[j] = ub[j] - x[j];
            dv[j] = -1.0;
        }
        if (g[j] > 0 && std::isfinite(lb[j])) {
            v[j] = x[j] - lb[j];
            dv[j] = 1.0;
        }
    }
}

bool in_bounds(const double* x, const double* lb, const double* ub) {
    for (int j = 0; j < NP; ++j)
        if (!(x[j] >= lb[j] && x[j] <= ub[j])) return false;
    return true;
}

// common.py step_size_to_bound: min step along s to a bound, hits = sign(s) where it is attained
double step_to_bound(const double* x, const double* s, const double* lb, const double* ub, int* hits) {
    double steps[NP], mn = INF;
    for (int j = 0; j < NP; ++j) {
        steps[j] = INF;
        if (s[j] != 0.0) steps[j] = std::max((lb[j] - x[j]) / s[j], (ub[j] - x[j]) / s[j]);
        mn = std::min(mn, steps[j]);
    }
    if (hits)
        for (int j = 0; j < NP; ++j) hits[j] = steps[j] == mn ? (s[j] > 0 ? 1 : s[j] < 0 ? -1 : 0) : 0;
    return mn;
}

// common.py intersect_trust_region: the two roots t of ||x + t s|| = Delta (t1 <= t2); false on the ValueErrors
bool intersect_tr(const double* x, const double* s, double Delta, double* t1, double* t2) {
    const double a = dot4(s, s);
    if (a == 0) return false;
    const double b = dot4(x, s);
    const double c = dot4(x, x) - Delta * Delta;
    if (c > 0) return false;
    const double d = std::sqrt(b * b - a * c);
    const double q = -(b + std::copysign(d, b));
    const double r1 = q / a, r2 = c / q;
    *t1 = std::min(r1, r2);
    *t2 = r1 < r2 ? r2 : r1;
    return true;
}

struct Quad {  // the scaled model: J_h [m][4], g_h, diag_h
    const double* Jh;
    int m;
    const double *gh, *diag;
    void Jdot(const double* s, double* out) const {
        for (int i = 0; i < m; ++i) out[i] = Jh[4 * i] * s[0] + Jh[4 * i + 1] * s[1] + Jh[4 * i + 2] * s[2] + Jh[4 * i + 3] * s[3];
    }
    // common.py evaluate_quadratic
    double eval(const double* s, double* tmp) const {
        Jdot(s, tmp);
        double q = 0.0;
        for (int i = 0; i < m; ++i) q += tmp[i] * tmp[i];
        for (int j = 0; j < NP; ++j) q += s[j] * diag[j] * s[j];
        return 0.5 * q + dot4(s, gh);
    }
    // common.py build_quadratic_1d (with s0 when given)
    void build1d(const double* s, const double* s0, double* tmp, double* tmp2, double* a, double* b, double* c) const {
        Jdot(s, tmp);
        double aa = 0.0;
        for (int i = 0; i < m; ++i) aa += tmp[i] * tmp[i];
        for (int j = 0; j < NP; ++j) aa += s[j] * diag[j] * s[j];
        aa *= 0.5;
        double bb = dot4(gh, s), cc = 0.0;
        if (s0) {
            Jdot(s0, tmp2);
            double uv = 0.0, uu = 0.0;
            for (int i = 0; i < m; ++i) {
                uv += tmp2[i] * tmp[i];
                uu += tmp2[i] * tmp2[i];
            }
            bb += uv;
            cc = 0.5 * uu + dot4(gh, s0);
            double ds = 0.0, d0 = 0.0;
            for (int j = 0; j < NP; ++j) {
                ds += s0[j] * diag[j] * s[j];
                d0 += s0[j] * diag[j] * s0[j];
            }
            bb += ds;
            cc += 0.5 * d0;
        }
        *a = aa;
        *b = bb;
        if (c) *c = cc;
    }
};

// common.py minimize_quadratic_1d: argmin of a t^2 + b t + c over [lb, ub] (first minimum of lb, ub, extremum)
void min_quad_1d(double a, double b, double lb, double ub, double c, double* tbest, double* ybest) {
    double t[3] = {lb, ub, 0.0};
    int nt = 2;
    if (a != 0) {
        const double ext = -0.5 * b / a;
        if (lb < ext && ext < ub) t[nt++] = ext;
    }
    int bi = 0;  // np.argmin: the first minimum, a NaN counting as the minimum
    double by = t[0] * (a * t[0] + b) + c;
    for (int i = 1; i < nt && !std::isnan(by); ++i) {
        const double y = t[i] * (a * t[i] + b) + c;
        if (y < by || std::isnan(y)) {
            by = y;
            bi = i;
        }
    }
    *tbest = t[bi];
    *ybest = by;
}

// SVD of the (m + 4) x 4 augmented matrix [J_h; diag(sqrt(diag_h))] as Householder QR + one-sided Jacobi on R.
// Returns s (descending), V (columns = right singular vectors, V[i][j] = component i of vector j) and
// uf = U^T f_aug.
void svd_aug(const double* Jh, int m, const double* diag_h, const double* f, std::vector<double>& A,
             std::vector<double>& fa, double* s, double V[NP][NP], double* uf) {
    const int M = m + NP;
    A.resize((size_t)M * NP);
    fa.resize(M);
    std::memcpy(A.data(), Jh, sizeof(double) * (size_t)m * NP);
    for (int i = 0; i < NP; ++i)
        for (int j = 0; j < NP; ++j) A[(size_t)(m + i) * NP + j] = i == j ? std::sqrt(diag_h[i]) : 0.0;
    std::memcpy(fa.data(), f, sizeof(double) * m);
    for (int i = 0; i < NP; ++i) fa[m + i] = 0.0;
    // Householder: A = Q R, fa <- Q^T fa
    for (int k = 0; k < NP; ++k) {
        double nrm = 0.0;
        for (int i = k; i < M; ++i) nrm += A[(size_t)i * NP + k] * A[(size_t)i * NP + k];
        nrm = std::sqrt(nrm);
        if (nrm == 0.0) continue;
        const double x0 = A[(size_t)k * NP + k];
        const double alpha = x0 > 0 ? -nrm : nrm;
        const double v0 = x0 - alpha;
        // v = (v0, A[k+1.., k]); v^T v = nrm^2 - x0^2 + v0^2
        const double vtv = nrm * nrm - x0 * x0 + v0 * v0;
        if (vtv == 0.0) continue;
        for (int j = k + 1; j < NP; ++j) {
            double d = v0 * A[(size_t)k * NP + j];
            for (int i = k + 1; i < M; ++i) d += A[(size_t)i * NP + k] * A[(size_t)i * NP + j];
            const double sc = 2.0 * d / vtv;
            A[(size_t)k * NP + j] -= sc * v0;
            for (int i = k + 1; i < M; ++i) A[(size_t)i * NP + j] -= sc * A[(size_t)i * NP + k];
        }
        double d = v0 * fa[k];
        for (int i = k + 1; i < M; ++i) d += A[(size_t)i * NP + k] * fa[i];
        const double sc = 2.0 * d / vtv;
        fa[k] -= sc * v0;
        for (int i = k + 1; i < M; ++i) fa[i] -= sc * A[(size_t)i * NP + k];
        A[(size_t)k * NP + k] = alpha;
        for (int i = k + 1; i < M; ++i) A[(size_t)i * NP + k] = 0.0;
    }
    // one-sided Jacobi on R (4 x 4): B = R V, columns orthogonalised
    double B[NP][NP], W[NP][NP];  // B[i][j]: row i, column j
    for (int i = 0; i < NP; ++i)
        for (int j = 0; j < NP; ++j) {
            B[i][j] = j >= i ? A[(size_t)i * NP + j] : 0.0;
            W[i][j] = i == j ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 60; ++sweep) {
        bool rotated = false;
        for (int p = 0; p < NP - 1; ++p)
            for (int q = p + 1; q < NP; ++q) {
                double al = 0.0, be = 0.0, ga = 0.0;
                for (int i = 0; i < NP; ++i) {
                    al += B[i][p] * B[i][p];
                    be += B[i][q] * B[i][q];
                    ga += B[i][p] * B[i][q];
                }
                if (ga == 0.0 || std::fabs(ga) <= 1e-17 * std::sqrt(al * be)) continue;
                rotated = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), sn = c * t;
                for (int i = 0; i < NP; ++i) {
                    const double bp = B[i][p], bq = B[i][q];
                    B[i][p] = c * bp - sn * bq;
                    B[i][q] = sn * bp + c * bq;
                    const double wp = W[i][p], wq = W[i][q];
                    W[i][p] = c * wp - sn * wq;
                    W[i][q] = sn * wp + c * wq;
                }
            }
        if (!rotated) break;
    }
    double sv[NP];
    int ord[NP];
    for (int j = 0; j < NP; ++j) {
        double n2 = 0.0;
        for (int i = 0; i < NP; ++i) n2 += B[i][j] * B[i][j];
        sv[j] = std::sqrt(n2);
        ord[j] = j;
    }
    std::stable_sort(ord, ord + NP, [&](int a, int b) { return sv[a] > sv[b]; });
    for (int jj = 0; jj < NP; ++jj) {
        const int j = ord[jj];
        s[jj] = sv[j];
        for (int i = 0; i < NP; ++i) V[i][jj] = W[i][j];
        double u = 0.0;
        if (sv[j] > 0.0) {
            for (int i = 0; i < NP; ++i) u += B[i][j] * fa[i];
            u /= sv[j];
        }
        uf[jj] = u;
    }
}

// common.py solve_lsq_trust_region (n = 4, m data rows): the regularised least-squares step of norm <= Delta
void solve_tr(int m, const double* uf, const double* s, const double V[NP][NP], double Delta, double* alpha_io,
              double* p) {
    double suf[NP];
    for (int j = 0; j < NP; ++j) suf[j] = s[j] * uf[j];
    auto phi_d = [&](double alpha, double* phi, double* dphi) {
        double pn = 0.0, sd = 0.0;
        for (int j = 0; j < NP; ++j) {
            const double den = s[j] * s[j] + alpha;
            pn += (suf[j] / den) * (suf[j] / den);
            sd += suf[j] * suf[j] / (den * den * den);
        }
        pn = std::sqrt(pn);
        *phi = pn - Delta;
        *dphi = -sd / pn;
    };
    const bool full_rank = m >= NP ? s[NP - 1] > EPS * m * s[0] : false;
    if (full_rank) {
        double c[NP];
        for (int j = 0; j < NP; ++j) c[j] = uf[j] / s[j];
        for (int i = 0; i < NP; ++i) p[i] = -(V[i][0] * c[0] + V[i][1] * c[1] + V[i][2] * c[2] + V[i][3] * c[3]);
        if (norm4(p) <= Delta) {
            *alpha_io = 0.0;
            return;
        }
    }
    double alpha_upper = norm4(suf) / Delta;
    double alpha_lower = 0.0;
    if (full_rank) {
        double phi, dphi;
        phi_d(0.0, &phi, &dphi);
        alpha_lower = -phi / dphi;
    }
    double alpha = *alpha_io;
    if (!full_rank && alpha == 0) alpha = std::max(0.001 * alpha_upper, std::sqrt(alpha_lower * alpha_upper));
    for (int it = 0; it < 10; ++it) {
        if (alpha < alpha_lower || alpha > alpha_upper) alpha = std::max(0.001 * alpha_upper, std::sqrt(alpha_lower * alpha_upper));
        double phi, dphi;
        phi_d(alpha, &phi, &dphi);
        if (phi < 0) alpha_upper = alpha;
        const double ratio = phi / dphi;
        alpha_lower = std::max(alpha_lower, alpha - ratio);
        alpha -= (phi + Delta) * ratio / Delta;
        if (std::fabs(phi) < 0.01 * Delta) break;
    }
    double c[NP];
    for (int j = 0; j < NP; ++j) c[j] = suf[j] / (s[j] * s[j] + alpha);
    for (int i = 0; i < NP; ++i) p[i] = -(V[i][0] * c[0] + V[i][1] * c[1] + V[i][2] * c[2] + V[i][3] * c[3]);
    const double sc = Delta / norm4(p);
    for (int i = 0; i < NP; ++i) p[i] *= sc;
    *alpha_io = alpha;
}

// trf.py select_step: the TRF step among the (reflected) trust-region step and the scaled anti-gradient;
// writes step, step_h, returns the predicted reduction
double select_step(const double* x, const Quad& Q, const double* d, const double* p_in, const double* ph_in,
                   double Delta, const double* lb, const double* ub, double theta, double* tmp, double* tmp2,
                   double* step, double* step_h) {
    double p[NP], p_h[NP];
    std::memcpy(p, p_in, sizeof(p));
    std::memcpy(p_h, ph_in, sizeof(p_h));
    double xp[NP];
    for (int j = 0; j < NP; ++j) xp[j] = x[j] + p[j];
    if (in_bounds(xp, lb, ub)) {
        const double pv = Q.eval(p_h, tmp);
        std::memcpy(step, p, sizeof(p));
        std::memcpy(step_h, p_h, sizeof(p_h));
        return -pv;
    }
    int hits[NP];
    const double p_stride = step_to_bound(x, p, lb, ub, hits);
    double r_h[NP], r[NP];
    for (int j = 0; j < NP; ++j) {
        r_h[j] = hits[j] != 0 ? -p_h[j] : p_h[j];
        r[j] = d[j] * r_h[j];
    }
    double x_on[NP];
    for (int j = 0; j < NP; ++j) {
        p[j] *= p_stride;
        p_h[j] *= p_stride;
        x_on[j] = x[j] + p[j];
    }
    double t1 = 0, to_tr = 0;
    if (!intersect_tr(p_h, r_h, Delta, &t1, &to_tr)) to_tr = 0.0;  // scipy raises here; never reached in practice
    const double to_bound = step_to_bound(x_on, r, lb, ub, nullptr);
    double r_stride = std::min(to_bound, to_tr), r_lo, r_up;
    if (r_stride > 0) {
        r_lo = (1 - theta) * p_stride / r_stride;
        r_up = r_stride == to_bound ? theta * to_bound : to_tr;
    } else {
        r_lo = 0;
        r_up = -1;
    }
    double r_value;
    if (r_lo <= r_up) {
        double a, b, c;
        Q.build1d(r_h, p_h, tmp, tmp2, &a, &b, &c);
        double rs;
        min_quad_1d(a, b, r_lo, r_up, c, &rs, &r_value);
        for (int j = 0; j < NP; ++j) {
            r_h[j] = r_h[j] * rs + p_h[j];
            r[j] = r_h[j] * d[j];
        }
    } else {
        r_value = INF;
    }
    for (int j = 0; j < NP; ++j) {
        p[j] *= theta;
        p_h[j] *= theta;
    }
    const double p_value = Q.eval(p_h, tmp);
    double ag_h[NP], ag[NP];
    for (int j = 0; j < NP; ++j) {
        ag_h[j] = -Q.gh[j];
        ag[j] = d[j] * ag_h[j];
    }
    const double to_tr2 = Delta / norm4(ag_h);
    const double to_b2 = step_to_bound(x, ag, lb, ub, nullptr);
    double ag_stride = to_b2 < to_tr2 ? theta * to_b2 : to_tr2;
    double a, b, ag_value;
    Q.build1d(ag_h, nullptr, tmp, tmp2, &a, &b, nullptr);
    min_quad_1d(a, b, 0, ag_stride, 0, &ag_stride, &ag_value);
    for (int j = 0; j < NP; ++j) {
        ag_h[j] *= ag_stride;
        ag[j] *= ag_stride;
    }
    if (p_value < r_value && p_value < ag_value) {
        std::memcpy(step, p, sizeof(p));
        std::memcpy(step_h, p_h, sizeof(p_h));
        return -p_value;
    } else if (r_value < p_value && r_value < ag_value) {
        std::memcpy(step, r, sizeof(r));
        std::memcpy(step_h, r_h, sizeof(r_h));
        return -r_value;
    }
    std::memcpy(step, ag, sizeof(ag));
    std::memcpy(step_h, ag_h, sizeof(ag_h));
    return -ag_value;
}

// common.py find_active_constraints + make_strictly_feasible
void make_strictly_feasible(double* x, const double* lb, const double* ub, double rstep) {
    for (int j = 0; j < NP; ++j) {
        int active = 0;
        if (rstep == 0) {
            if (x[j] <= lb[j]) active = -1;
            if (x[j] >= ub[j]) active = 1;
        } else {
            const double ld = x[j] - lb[j], ud = ub[j] - x[j];
            const double lt = rstep * std::max(1.0, std::fabs(lb[j])), ut = rstep * std::max(1.0, std::fabs(ub[j]));
            if (std::isfinite(lb[j]) && ld <= std::min(ud, lt)) active = -1;
            if (std::isfinite(ub[j]) && ud <= std::min(ld, ut)) active = 1;
        }
        double xn = x[j];
        if (active == -1) xn = rstep == 0 ? std::nextafter(lb[j], ub[j]) : lb[j] + rstep * std::max(1.0, std::fabs(lb[j]));
        if (active == 1) xn = rstep == 0 ? std::nextafter(ub[j], lb[j]) : ub[j] - rstep * std::max(1.0, std::fabs(ub[j]));
        if (xn < lb[j] || xn > ub[j]) xn = 0.5 * (lb[j] + ub[j]);
        x[j] = xn;
    }
}

// trf.py trf_bounds (x_scale = 1, loss soft_l1, tr_solver 'exact')
int fit_one(const Problem& P, double* x_out) {
    const int m = P.m;
    const double *lb = P.lb, *ub = P.ub;
    std::vector<double> J((size_t)m * NP), f(m), fnew(m), tmp(m), tmp2(m), Jh((size_t)m * NP), Aw, fw;
    double x[NP] = {1.0, 1.0, 1.0, 1.0};
    make_strictly_feasible(x, lb, ub, 1e-10);
    P.fun(x, f.data());
    int nfev = 1;
    P.jac(x, J.data());
    double cost = robust_scale(J.data(), f.data(), m);
    double g[NP], v[NP], dv[NP];
    grad(J.data(), f.data(), m, g);
    cl_scaling(x, g, lb, ub, v, dv);
    double xs[NP];
    for (int j = 0; j < NP; ++j) xs[j] = x[j] / std::sqrt(v[j]);
    double Delta = norm4(xs);
    if (Delta == 0) Delta = 1.0;
    double alpha = 0.0;
    int status = -1;
    for (;;) {
        cl_scaling(x, g, lb, ub, v, dv);
        double g_norm = 0.0;
        for (int j = 0; j < NP; ++j) g_norm = std::max(g_norm, std::fabs(g[j] * v[j]));
        if (g_norm < GTOL) status = 1;
        if (status != -1 || nfev == MAX_NFEV) break;
        double d[NP], diag_h[NP], g_h[NP];
        for (int j = 0; j < NP; ++j) {
            d[j] = std::sqrt(v[j]);
            diag_h[j] = g[j] * dv[j];
            g_h[j] = d[j] * g[j];
        }
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < NP; ++j) Jh[(size_t)i * NP + j] = J[(size_t)i * NP + j] * d[j];
        double s[NP], V[NP][NP], uf[NP];
        svd_aug(Jh.data(), m, diag_h, f.data(), Aw, fw, s, V, uf);
        const double theta = std::max(0.995, 1 - g_norm);
        const Quad Q{Jh.data(), m, g_h, diag_h};
        double actual_reduction = -1, cost_new = 0.0, xnew[NP];
        while (actual_reduction <= 0 && nfev < MAX_NFEV) {
            double p_h[NP], p[NP], step[NP], step_h[NP];
            solve_tr(m, uf, s, V, Delta, &alpha, p_h);
            for (int j = 0; j < NP; ++j) p[j] = d[j] * p_h[j];
            const double predicted = select_step(x, Q, d, p, p_h, Delta, lb, ub, theta, tmp.data(), tmp2.data(), step, step_h);
            for (int j = 0; j < NP; ++j) xnew[j] = x[j] + step[j];
            make_strictly_feasible(xnew, lb, ub, 0.0);
            P.fun(xnew, fnew.data());
            ++nfev;
            const double step_h_norm = norm4(step_h);
            bool finite = true;
            for (int i = 0; i < m; ++i) finite = finite && std::isfinite(fnew[i]);
            if (!finite) {
                Delta = 0.25 * step_h_norm;
                continue;
            }
            cost_new = cost_only(fnew.data(), m);
            actual_reduction = cost - cost_new;
            // update_tr_radius
            double ratio;
            if (predicted > 0) ratio = actual_reduction / predicted;
            else if (predicted == actual_reduction && predicted == 0) ratio = 1;
            else ratio = 0;
            double Delta_new = Delta;
            if (ratio < 0.25) Delta_new = 0.25 * step_h_norm;
            else if (ratio > 0.75 && step_h_norm > 0.95 * Delta) Delta_new = Delta * 2.0;
            // check_termination
            const double step_norm = norm4(step);
            const bool ftol_ok = actual_reduction < FTOL * cost && ratio > 0.25;
            const bool xtol_ok = step_norm < XTOL * (XTOL + norm4(x));
            if (ftol_ok || xtol_ok) {
                status = ftol_ok && xtol_ok ? 4 : ftol_ok ? 2 : 3;
                break;
            }
            alpha *= Delta / Delta_new;
            Delta = Delta_new;
        }
        if (actual_reduction > 0) {
            std::memcpy(x, xnew, sizeof(x));
            std::swap(f, fnew);
            cost = cost_new;
            P.jac(x, J.data());
            robust_scale(J.data(), f.data(), m);
            grad(J.data(), f.data(), m, g);
        }
    }
    std::memcpy(x_out, x, sizeof(x));
    return nfev;
}

// ===================================================================================== Pareto primitives
inline bool dominates(const double* a, const double* b, int k) {  // a >= b everywhere and > somewhere
    bool gt = false;
    for (int j = 0; j < k; ++j) {
        if (!(a[j] >= b[j])) return false;
        gt = gt || a[j] > b[j];
    }
    return gt;
}

// area of the union of boxes [0, x] x [0, y] (points >= 0)
double area2d(std::vector<std::pair<double, double>>& pts) {
    std::sort(pts.begin(), pts.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    double area = 0.0, ymax = 0.0;
    for (size_t i = 0; i < pts.size(); ++i) {
        ymax = std::max(ymax, pts[i].second);
        const double xn = i + 1 < pts.size() ? pts[i + 1].first : 0.0;
        area += (pts[i].first - xn) * ymax;
    }
    return area;
}

// dominated volume of points (all >= 0 already), k in {1, 2, 3}; slices along the last axis
double volume(const std::vector<double>& f, int n, int k) {
    if (n == 0) return 0.0;
    if (k == 1) {
        double mx = f[0];
        for (int i = 1; i < n; ++i) mx = std::max(mx, f[i]);
        return mx;
    }
    std::vector<std::pair<double, double>> pts;
    pts.reserve(n);
    if (k == 2) {
        for (int i = 0; i < n; ++i) pts.emplace_back(f[2 * i], f[2 * i + 1]);
        return area2d(pts);
    }
    std::vector<int> ord(n);
    for (int i = 0; i < n; ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return f[3 * a + 2] > f[3 * b + 2]; });
    // incremental staircase: after adding the i-th highest point, the slab (z_{i+1}, z_i] has the prefix's area
    std::vector<std::pair<double, double>> stair;  // non-dominated (x asc, y desc)
    double vol = 0.0, area = 0.0;
    for (int ii = 0; ii < n; ++ii) {
        const int i = ord[ii];
        const double px = f[3 * i], py = f[3 * i + 1];
        bool covered = false;
        for (const auto& q : stair)
            if (q.first >= px && q.second >= py) {
                covered = true;
                break;
            }
        if (!covered) {
            std::vector<std::pair<double, double>> ns;
            ns.reserve(stair.size() + 1);
            for (const auto& q : stair)
                if (!(px >= q.first && py >= q.second)) ns.push_back(q);
            ns.emplace_back(px, py);
            std::sort(ns.begin(), ns.end());
            stair.swap(ns);
            pts.assign(stair.begin(), stair.end());
            area = area2d(pts);
        }
        const double z = f[3 * i + 2];
        const double zn = ii + 1 < n ? f[3 * ord[ii + 1] + 2] : 0.0;
        if (z > zn) vol += (z - zn) * area;
    }
    return vol;
}

double round4(double v) {  // Python round(v, 4): correctly rounded decimal, ties to even
    if (!std::isfinite(v)) return v;
    char buf[64];
    snprintf(buf, sizeof(buf), "%.4f", v);  // glibc: exact decimal expansion, round-half-even
    return std::strtod(buf, nullptr);
}

double hypervolume_pts(const double* objs, int64_t n, int k) {
    std::vector<double> f;
    f.reserve((size_t)n * k);
    int cnt = 0;
    bool nan = false;
    for (int64_t i = 0; i < n; ++i) {
        bool ok = true;
        for (int j = 0; j < k; ++j) {
            if (std::isnan(objs[i * k + j])) nan = true;
            ok = ok && objs[i * k + j] >= 0;
        }
        if (ok) {
            f.insert(f.end(), objs + i * k, objs + (i + 1) * k);
            ++cnt;
        }
    }
    if (nan) return std::nan("");  // InnerHyperVolume keeps NaN points and returns NaN
    return round4(volume(f, cnt, k));
}

// utils.compute_sparsity: per objective, sorted values, squared steps summed in that order
double sparsity_nd(const std::vector<double>& e, int n, int k, std::vector<double>& col) {
    if (n < 2) return 0.0;
    double sp = 0.0;
    col.resize(n);
    for (int d = 0; d < k; ++d) {
        for (int i = 0; i < n; ++i) col[i] = e[(size_t)i * k + d];
        std::sort(col.begin(), col.end());
        for (int i = 1; i < n; ++i) sp += (col[i] - col[i - 1]) * (col[i] - col[i - 1]);
    }
    return sp / (double)(n - 1);
}

// utils.update_ep: drop points the new one weakly dominates, insert it before the first larger obj0 unless an
// archive point beats it by more than 1e-5
void update_ep(const std::vector<double>& ep, int n, const double* x, int k, std::vector<double>& out, int* nout) {
    out.clear();
    bool neg = false;
    for (int j = 0; j < k; ++j) neg = neg || x[j] < 0;
    if (neg) {
        out = ep;
        *nout = n;
        return;
    }
    bool on_ep = true;
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        const double* q = &ep[(size_t)i * k];
        bool dom = true, ge = true, gt = false;
        for (int j = 0; j < k; ++j) {
            dom = dom && x[j] >= q[j];
            ge = ge && q[j] >= x[j] - 1e-5;
            gt = gt || q[j] > x[j] + 1e-5;
        }
        if (ge && gt) on_ep = false;
        if (!dom) {
            out.insert(out.end(), q, q + k);
            ++cnt;
        }
    }
    if (on_ep) {
        int pos = cnt;
        for (int i = 0; i < cnt; ++i)
            if (x[0] < out[(size_t)i * k]) {
                pos = i;
                break;
            }
        out.insert(out.begin() + (size_t)pos * k, x, x + k);
        ++cnt;
    }
    *nout = cnt;
}

// 2-D: EP indices of (virtual EP + [x]) in obj0 order.  The virtual EP is itself a front (mutually
// non-dominated, >= 0, obj0 ascending), so only x's relations matter; kept points with equal obj0 are exact
// duplicates, whose order does not change any value below.
void merge_2d(const std::vector<double>& ep, int n, const double* x, std::vector<double>& out, int* nout) {
    out.clear();
    bool x_keep = x[0] >= 0 && x[1] >= 0;
    for (int i = 0; i < n && x_keep; ++i)
        if (dominates(&ep[2 * i], x, 2)) x_keep = false;
    int cnt = 0;
    bool placed = !x_keep;
    for (int i = 0; i < n; ++i) {
        const double* q = &ep[2 * i];
        if (!placed && x[0] < q[0]) {
            out.push_back(x[0]);
            out.push_back(x[1]);
            ++cnt;
            placed = true;
        }
        if (dominates(x, q, 2)) continue;
        out.push_back(q[0]);
        out.push_back(q[1]);
        ++cnt;
    }
    if (!placed) {
        out.push_back(x[0]);
        out.push_back(x[1]);
        ++cnt;
    }
    *nout = cnt;
}

// population_2d.py:185-202 on a front already in obj0 order
void score_2d(const std::vector<double>& e, int n, double* hv_out, double* sp_out) {
    double hv = 0.0, xp = 0.0;
    for (int i = 0; i < n; ++i) {
        hv += (std::max(0.0, e[2 * i]) - xp) * (std::max(0.0, e[2 * i + 1]) - 0.0);
        xp = std::max(0.0, e[2 * i]);
    }
    double sp = 0.0;
    if (n >= 2) {
        for (int i = 1; i < n; ++i) {
            const double a = e[2 * i] - e[2 * i - 2], b = e[2 * i + 1] - e[2 * i - 1];
            sp += a * a + b * b;
        }
        sp /= (double)(n - 1);
    }
    *hv_out = hv;
    *sp_out = sp;
}

}  // namespace

extern "C" {

int pgm_host_abi_version(void) { return PGM_HOST_ABI_VERSION; }
const char* pgm_host_last_error(void) { return g_err; }

int pgm_fit_hyperbolic(int64_t nfit, const int64_t* off, const double* x, const double* y, const double* w,
                       const double* a_hi, double* params, int32_t* nfev, int nthreads) {
    if (nfit < 0 || (nfit > 0 && (!off || !x || !y || !w || !a_hi || !params)))
        return fail(E_INVALID_ARG, "pgm_fit_hyperbolic: null buffer");
    for (int64_t i = 0; i < nfit; ++i) {
        if (off[i + 1] <= off[i]) return fail(E_INVALID_ARG, "pgm_fit_hyperbolic: problem %lld has no rows", (long long)i);
        if (!(a_hi[i] > 0)) return fail(E_INVALID_ARG, "pgm_fit_hyperbolic: upper bound of A must exceed 0");
    }
    parallel_for(nfit, resolve_threads(nthreads, nfit), [&](int64_t i) {
        Problem P{(int)(off[i + 1] - off[i]), x + off[i], y + off[i], w + off[i], {0.0, 0.1, -5.0, -500.0},
                  {a_hi[i], 20.0, 5.0, 500.0}};
        const int ne = fit_one(P, params + 4 * i);
        if (nfev) nfev[i] = ne;
    });
    return 0;
}

int pgm_ep_mask(int64_t n, int k, const double* objs, uint8_t* keep) {
    if (n < 0 || k < 1 || (n > 0 && (!objs || !keep))) return fail(E_INVALID_ARG, "pgm_ep_mask: bad arguments");
    for (int64_t i = 0; i < n; ++i) {
        bool ok = true;
        for (int j = 0; j < k; ++j) ok = ok && objs[i * k + j] >= 0;
        for (int64_t q = 0; q < n && ok; ++q)
            if (dominates(objs + q * k, objs + i * k, k)) ok = false;
        keep[i] = ok ? 1 : 0;
    }
    return 0;
}

int pgm_hypervolume(int64_t n, int k, const double* objs, double* hv) {
    if (n < 0 || k < 1 || k > 3 || !hv || (n > 0 && !objs)) return fail(E_INVALID_ARG, "pgm_hypervolume: bad arguments (k in 1..3)");
    *hv = hypervolume_pts(objs, n, k);
    return 0;
}

int pgm_select_greedy(int k, int mode, int64_t n_ep, const double* ep, int64_t n_cand, const double* preds,
                      double alpha, int n_pick, int nthreads, int32_t* picks, int32_t* n_picked) {
    if (k < 2 || k > 3 || (mode != PGM_SELECT_STAIRCASE && mode != PGM_SELECT_UPDATE_EP) ||
        (mode == PGM_SELECT_STAIRCASE && k != 2) || n_ep < 0 || n_cand < 0 || n_pick < 0 || !n_picked ||
        (n_pick > 0 && !picks) || (n_ep > 0 && !ep) || (n_cand > 0 && !preds))
        return fail(E_INVALID_ARG, "pgm_select_greedy: bad arguments (k in 2..3, staircase mode needs k = 2)");
    const bool stair = mode == PGM_SELECT_STAIRCASE;
    std::vector<double> vep(ep, ep + n_ep * k);
    int nv = (int)n_ep;
    std::vector<uint8_t> avail(n_cand, 1);
    std::vector<double> score(n_cand);
    const int nt = stair ? 1 : resolve_threads(nthreads, n_cand);
    *n_picked = 0;
    for (int r = 0; r < n_pick; ++r) {
        parallel_for(n_cand, nt, [&](int64_t c) {
            if (!avail[c]) return;
            thread_local std::vector<double> e, col;
            int ne = 0;
            double hv, sp;
            if (stair) {
                merge_2d(vep, nv, preds + 2 * c, e, &ne);
                score_2d(e, ne, &hv, &sp);
            } else {
                update_ep(vep, nv, preds + k * c, k, e, &ne);
                hv = ne ? hypervolume_pts(e.data(), ne, k) : 0.0;
                sp = ne ? sparsity_nd(e, ne, k, col) : 0.0;
            }
            score[c] = hv - alpha * sp;
        });
        int64_t best = -1;
        double bv = -INF;
        for (int64_t c = 0; c < n_cand; ++c)
            if (avail[c] && score[c] > bv) {
                bv = score[c];
                best = c;
            }
        if (best < 0) break;
        picks[r] = (int32_t)best;
        ++*n_picked;
        avail[best] = 0;
        std::vector<double> e;
        int ne = 0;
        if (stair) merge_2d(vep, nv, preds + 2 * best, e, &ne);
        else update_ep(vep, nv, preds + k * best, k, e, &ne);
        vep.swap(e);
        nv = ne;
    }
    return 0;
}

}  // extern "C"
