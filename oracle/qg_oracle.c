/*
 * CPU ORACLE -- test infrastructure only, never part of the product path.
 *
 * Plain-C (OpenMP) restatement of the reference hot path
 * (JSLeadbetter/julia-ocean-modelling @ 2024-10-08), used
 *   (a) by tests/ as the checker at sizes where the scipy oracle (qg_ref.py) is too slow,
 *   (b) by bench.py's cpu_baseline leg ("kind": "port").
 * It is itself pinned to oracle/qg_ref.py (and through it to the reference's own known
 * answers) by tests/test_oracle_c.py.
 *
 * Layout: Julia column-major (M+2, P+2) fields, element (i, j) at i + (M+2)*j, one ghost
 * ring; state arrays (M+2, P+2, 2, 3) with slot 0 newest.
 *
 * Stencils follow the reference term by term (build with -ffp-contract=off):
 *   laplace_5p      src/schemes/laplacian.jl:15-27
 *   cd              src/model.jl:68-80
 *   j_pp/j_pt/j_tp  src/schemes/arakawa.jl:7-56,  J  arakawa.jl:58-62
 *   ghost fill      src/schemes/boundary_conditions.jl:2-13
 *   zeta_f1/2       src/model.jl:139-153; Euler/AB3 model.jl:123-136; evolve model.jl:155-170
 *   evolve_psi!     src/model.jl:172-199 (P_matrix(H_1,H_1) by default)
 * The CHOLMOD solves (model.jl:186,191) are replaced by an exact periodic DFT solve of the
 * same operator (construct_spA, laplacian.jl:54-58); the pinned Poisson system
 * (laplacian.jl:66-75, b[1]=0) is reproduced exactly: adjust the RHS at interior (1,1) by
 * -sum(f) (which makes it compatible), solve mean-free, subtract the value at (1,1).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    double H_1, H_2, beta, Lx, Ly, dt, T, U, dx, visc, r, R_d, initial_kick;
    long M, P;
    double Pfwd[4]; /* back-projection matrix, row-major [[p11,p12],[p21,p22]] */
    /* wind-forcing extension (not in the reference; include/qg_mi355.h qg_params): 0 = off */
    double wind_tau0, wind_rho0;
} qgo_params;

/* the extension's upper-layer forcing at global interior row jg (0-based) of P_total rows;
 * the same expression as the device library's host table (qg_common.hpp wind_row) */
static double wind_row(double tau0, double rho0, double H1, double dx, long P_total, long jg) {
    const double pi2 = 6.283185307179586;
    const double A = (pi2 * tau0) / (rho0 * H1 * ((double)P_total * dx));
    return -A * sin(pi2 * (((double)jg + 0.5) / (double)P_total));
}

#define IDX(i, j, M2) ((size_t)(i) + (size_t)(M2) * (size_t)(j))

/* ---------------------------------------------------------------- params */
static double ratio_term(const qgo_params *m) {
    return 0.5 * (m->H_1 + m->H_2) / ((m->R_d * m->R_d) * ((1 / m->H_1) + (1 / m->H_2)));
}
static double S1_plus(const qgo_params *m) { return (2 * ratio_term(m)) / (m->H_1 * (m->H_1 + m->H_2)); }
static double S2_minus(const qgo_params *m) { return (2 * ratio_term(m)) / (m->H_2 * (m->H_1 + m->H_2)); }
static double beta_1(const qgo_params *m) { return m->beta + (S1_plus(m) * m->U); }
static double beta_2(const qgo_params *m) { return m->beta - (S2_minus(m) * m->U); }
static double S_eig(const qgo_params *m) { return -1 / (m->R_d * m->R_d); }

/* ---------------------------------------------------------------- ghosts */
void qgo_fill_ghosts(double *b, long M2, long P2) {
    for (long i = 1; i < M2 - 1; ++i) {
        b[IDX(i, 0, M2)] = b[IDX(i, P2 - 2, M2)];
        b[IDX(i, P2 - 1, M2)] = b[IDX(i, 1, M2)];
    }
    for (long j = 1; j < P2 - 1; ++j) {
        b[IDX(0, j, M2)] = b[IDX(M2 - 2, j, M2)];
        b[IDX(M2 - 1, j, M2)] = b[IDX(1, j, M2)];
    }
    b[IDX(0, 0, M2)] = b[IDX(M2 - 2, P2 - 2, M2)];
    b[IDX(0, P2 - 1, M2)] = b[IDX(M2 - 2, 1, M2)];
    b[IDX(M2 - 1, P2 - 1, M2)] = b[IDX(1, 1, M2)];
    b[IDX(M2 - 1, 0, M2)] = b[IDX(1, P2 - 2, M2)];
}

/* ---------------------------------------------------------------- stencils */
void qgo_laplace_5p(const double *u, double *lap, long M2, long P2, double dx) {
    const double idx = 1.0 / dx, idx2 = idx * idx;
#pragma omp parallel for schedule(static)
    for (long j = 1; j < P2 - 1; ++j)
        for (long i = 1; i < M2 - 1; ++i)
            lap[IDX(i, j, M2)] = ((((u[IDX(i - 1, j, M2)] + u[IDX(i + 1, j, M2)]) - 4 * u[IDX(i, j, M2)])
                                   + u[IDX(i, j - 1, M2)]) + u[IDX(i, j + 1, M2)]) * idx2;
    qgo_fill_ghosts(lap, M2, P2);
}

void qgo_cd(const double *u, double *out, long M2, long P2, double dx) {
    const double c = 0.5 * (1.0 / dx);
#pragma omp parallel for schedule(static)
    for (long j = 1; j < P2 - 1; ++j)
        for (long i = 1; i < M2 - 1; ++i)
            out[IDX(i, j, M2)] = c * (u[IDX(i + 1, j, M2)] - u[IDX(i - 1, j, M2)]);
    qgo_fill_ghosts(out, M2, P2);
}

void qgo_J(double dx, const double *z, const double *p, double *out, long M2, long P2) {
    const double den = 12 * (dx * dx);
#pragma omp parallel for schedule(static)
    for (long j = 1; j < P2 - 1; ++j)
        for (long i = 1; i < M2 - 1; ++i) {
#define Z(a, b) z[IDX(i + (a), j + (b), M2)]
#define PS(a, b) p[IDX(i + (a), j + (b), M2)]
            double jpp = (Z(1, 0) - Z(-1, 0)) * (PS(0, 1) - PS(0, -1))
                       - (Z(0, 1) - Z(0, -1)) * (PS(1, 0) - PS(-1, 0));
            double jpt = ((Z(1, 0) * (PS(1, 1) - PS(1, -1)) - Z(-1, 0) * (PS(-1, 1) - PS(-1, -1)))
                          - Z(0, 1) * (PS(1, 1) - PS(-1, 1)))
                         + Z(0, -1) * (PS(1, -1) - PS(-1, -1));
            double jtp = ((Z(1, 1) * (PS(0, 1) - PS(1, 0)) - Z(-1, -1) * (PS(-1, 0) - PS(0, -1)))
                          - Z(-1, 1) * (PS(0, 1) - PS(-1, 0)))
                         + Z(1, -1) * (PS(1, 0) - PS(0, -1));
            out[IDX(i, j, M2)] = ((jpp + jpt) + jtp) / den;
#undef Z
#undef PS
        }
    qgo_fill_ghosts(out, M2, P2);
}

/* ---------------------------------------------------------------- seeded ICs */
static inline double u01(uint64_t seed, uint64_t k) {
    uint64_t x = seed + (k + 1) * 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    x = x ^ (x >> 31);
    return (double)(x >> 11) * 0x1.0p-53;
}

/* model.jl:37-62 with seeded noise; zeta/psi (M+2,P+2,2,3) are zeroed first */
void qgo_initialise(const qgo_params *m, uint64_t seed1, uint64_t seed2, double *zeta, double *psi) {
    const long M2 = m->M + 2, P2 = m->P + 2;
    const size_t F = (size_t)M2 * P2;
    memset(zeta, 0, sizeof(double) * F * 6);
    memset(psi, 0, sizeof(double) * F * 6);
    const double amp = m->initial_kick * m->U * m->Ly;
    double *p1 = psi, *p2 = psi + F; /* [:,:,layer,slot0] */
    for (long j = 0; j < m->P; ++j)
        for (long i = 0; i < m->M; ++i) {
            uint64_t k = (uint64_t)i + (uint64_t)m->M * (uint64_t)j;
            p1[IDX(i + 1, j + 1, M2)] = amp * u01(seed1, k);
            p2[IDX(i + 1, j + 1, M2)] = amp * u01(seed2, k);
        }
    qgo_fill_ghosts(p1, M2, P2);
    qgo_fill_ghosts(p2, M2, P2);
    double *l1 = malloc(sizeof(double) * F), *l2 = malloc(sizeof(double) * F);
    qgo_laplace_5p(p1, l1, M2, P2, m->dx);
    qgo_laplace_5p(p2, l2, M2, P2, m->dx);
    const double s1 = S1_plus(m), s2 = S2_minus(m);
    for (size_t q = 0; q < F; ++q) {
        zeta[q] = l1[q] + s1 * (p2[q] - p1[q]);
        zeta[F + q] = l2[q] + s2 * (p1[q] - p2[q]);
    }
    qgo_fill_ghosts(zeta, M2, P2);
    qgo_fill_ghosts(zeta + F, M2, P2);
    free(l1);
    free(l2);
}

/* ---------------------------------------------------------------- tendency */
/* zeta_f1 / zeta_f2 (model.jl:139-153) for one layer; all arrays (M+2,P+2) */
static void rhs(const qgo_params *m, int layer, const double *z, const double *p, double *f, double *t1,
                double *t2, double *t3) {
    const long M2 = m->M + 2, P2 = m->P + 2;
    const size_t F = (size_t)M2 * P2;
    qgo_laplace_5p(p, t1, M2, P2, m->dx);  /* lap(psi)          */
    qgo_laplace_5p(t1, t2, M2, P2, m->dx); /* lap(lap(psi))     */
    qgo_J(m->dx, z, p, t3, M2, P2);        /* J(zeta, psi)      */
    /* f = visc*t2 - t3 - beta_l*cd(psi) - (layer1: U*cd(zeta) | layer2: r*lap(psi)) */
    double *cdp = malloc(sizeof(double) * F), *x = malloc(sizeof(double) * F);
    qgo_cd(p, cdp, M2, P2, m->dx);
    const double bl = layer == 0 ? beta_1(m) : beta_2(m);
    if (layer == 0) {
        qgo_cd(z, x, M2, P2, m->dx);
        for (size_t q = 0; q < F; ++q)
            f[q] = ((m->visc * t2[q] - t3[q]) - bl * cdp[q]) - m->U * x[q];
        if (m->wind_tau0 != 0) /* extension: + w_j, ghost rows take their periodic image */
            for (long j = 0; j < P2; ++j) {
                const long jj = (j - 1 + m->P) % m->P;
                const double w = wind_row(m->wind_tau0, m->wind_rho0, m->H_1, m->dx, m->P, jj);
                for (long i = 0; i < M2; ++i) f[IDX(i, j, M2)] = f[IDX(i, j, M2)] + w;
            }
    } else {
        for (size_t q = 0; q < F; ++q)
            f[q] = ((m->visc * t2[q] - t3[q]) - bl * cdp[q]) - m->r * t1[q];
    }
    free(cdp);
    free(x);
}

static void shift3(double *arr, long layer, size_t F, const double *newv) {
    /* store_new_state! (model.jl:102-106); arr is (M+2,P+2,2,3) */
    double *s0 = arr + F * (layer + 0), *s1 = arr + F * (layer + 2), *s2 = arr + F * (layer + 4);
    memcpy(s2, s1, sizeof(double) * F);
    memcpy(s1, s0, sizeof(double) * F);
    memcpy(s0, newv, sizeof(double) * F);
}

void qgo_evolve_zeta(const qgo_params *m, double *zeta, const double *psi, long timestep, double *f_store) {
    const size_t F = (size_t)(m->M + 2) * (m->P + 2);
    double *f1 = malloc(sizeof(double) * F), *nz = malloc(sizeof(double) * F);
    double *t1 = malloc(sizeof(double) * F), *t2 = malloc(sizeof(double) * F), *t3 = malloc(sizeof(double) * F);
    for (int l = 0; l < 2; ++l) {
        const double *z = zeta + F * l, *p = psi + F * l;
        rhs(m, l, z, p, f1, t1, t2, t3);
        shift3(f_store, l, F, f1);
        if (timestep == 1 || timestep == 2) {
            for (size_t q = 0; q < F; ++q) nz[q] = z[q] + (m->dt * f1[q]);
        } else {
            const double *fa = f_store + F * (l + 2), *fb = f_store + F * (l + 4);
            for (size_t q = 0; q < F; ++q)
                nz[q] = z[q] + m->dt * ((((23.0 / 12.0) * f1[q]) - ((16.0 / 12.0) * fa[q])) + ((5.0 / 12.0) * fb[q]));
        }
        shift3(zeta, l, F, nz);
    }
    free(f1); free(nz); free(t1); free(t2); free(t3);
}

/* ---------------------------------------------------------------- exact periodic solve */
typedef struct { double re, im; } cplx;

static int is_pow2(long n) { return n > 0 && (n & (n - 1)) == 0; }

/* in-place complex DFT of length n (sign -1 forward, +1 inverse, unnormalised) */
static void dft_line(cplx *a, long n, int sign, cplx *work) {
    if (is_pow2(n)) {
        for (long i = 1, j = 0; i < n; ++i) { /* bit reversal */
            long bit = n >> 1;
            for (; j & bit; bit >>= 1) j ^= bit;
            j ^= bit;
            if (i < j) { cplx t = a[i]; a[i] = a[j]; a[j] = t; }
        }
        for (long len = 2; len <= n; len <<= 1) {
            long h = len >> 1;
            for (long k = 0; k < h; ++k) {
                double ang = sign * 2.0 * M_PI * (double)k / (double)len;
                double wr = cos(ang), wi = sin(ang);
                for (long s = 0; s < n; s += len) {
                    cplx u = a[s + k], v = a[s + k + h];
                    double vr = v.re * wr - v.im * wi, vi = v.re * wi + v.im * wr;
                    a[s + k].re = u.re + vr; a[s + k].im = u.im + vi;
                    a[s + k + h].re = u.re - vr; a[s + k + h].im = u.im - vi;
                }
            }
        }
    } else { /* naive DFT for small non-power-of-two sizes */
        for (long k = 0; k < n; ++k) {
            double sr = 0, si = 0;
            for (long q = 0; q < n; ++q) {
                double ang = sign * 2.0 * M_PI * (double)((k * q) % n) / (double)n;
                double c = cos(ang), s = sin(ang);
                sr += a[q].re * c - a[q].im * s;
                si += a[q].re * s + a[q].im * c;
            }
            work[k].re = sr; work[k].im = si;
        }
        memcpy(a, work, sizeof(cplx) * n);
    }
}

static void dft2(cplx *g, long M, long P, int sign) {
#pragma omp parallel
    {
        cplx *w = malloc(sizeof(cplx) * (M > P ? M : P));
        cplx *col = malloc(sizeof(cplx) * P);
#pragma omp for schedule(static)
        for (long j = 0; j < P; ++j) dft_line(g + (size_t)M * j, M, sign, w);
#pragma omp for schedule(static)
        for (long i = 0; i < M; ++i) {
            for (long j = 0; j < P; ++j) col[j] = g[i + (size_t)M * j];
            dft_line(col, P, sign, w);
            for (long j = 0; j < P; ++j) g[i + (size_t)M * j] = col[j];
        }
        free(w);
        free(col);
    }
}

/*
 * Solve construct_spA(M,P,dx,alpha) x = f over the interior of the (M+2,P+2) field f,
 * i.e. the same x the reference gets from `cholesky(-A) \ -vec(f)`; pinned != 0 selects the
 * pinned Poisson system of get_poisson_cholesky (alpha must be 0).  out gets ghosts.
 */
int qgo_solve(long M, long P, double dx, double alpha, int pinned, const double *f, double *out) {
    const long M2 = M + 2;
    if (M < 1 || P < 1) return -2;
    cplx *g = malloc(sizeof(cplx) * (size_t)M * P);
    if (!g) return -1;
    double sum = 0, comp = 0; /* (compensated: the compatibility shift of up to 1e9 terms) */
    for (long j = 0; j < P; ++j)
        for (long i = 0; i < M; ++i) {
            double v = f[IDX(i + 1, j + 1, M2)];
            g[i + (size_t)M * j].re = v;
            g[i + (size_t)M * j].im = 0;
            const double y = v - comp, t = sum + y;
            comp = (t - sum) - y;
            sum = t;
        }
    if (pinned) g[0].re -= sum; /* compatible RHS: f'(1,1) = -sum_{k != 1} f_k */
    dft2(g, M, P, -1);
    const double idx = 1.0 / dx, idx2 = idx * idx;
    /* eigenvalues of the periodic [1 -2 1] in the cancellation-free form 2 cos(t) - 2 =
     * -4 sin^2(t / 2): the form 2 cos(t) + 2 cos(s) - 4 loses the gravest modes' eigenvalues to
     * cancellation (absolute error ~eps against (2 pi / P)^2: 2e-9 relative psi error on a
     * 256 x 32768 Poisson problem against a long-double solve, tools/r06/solve_precision.py) */
    double *sx = malloc(sizeof(double) * (size_t)M), *sy = malloc(sizeof(double) * (size_t)P);
    for (long k = 0; k < M; ++k) { const double t = sin(M_PI * (double)k / (double)M); sx[k] = t * t; }
    for (long k = 0; k < P; ++k) { const double t = sin(M_PI * (double)k / (double)P); sy[k] = t * t; }
    for (long ky = 0; ky < P; ++ky)
        for (long kx = 0; kx < M; ++kx) {
            double lam = idx2 * (-4 * (sx[kx] + sy[ky])) + alpha;
            cplx *c = &g[kx + (size_t)M * ky];
            if (pinned && kx == 0 && ky == 0) { c->re = 0; c->im = 0; continue; }
            c->re /= lam; c->im /= lam;
        }
    free(sx);
    free(sy);
    dft2(g, M, P, +1);
    const double inv = 1.0 / ((double)M * (double)P);
    const double shift = pinned ? g[0].re * inv : 0.0;
    for (long j = 0; j < P; ++j)
        for (long i = 0; i < M; ++i) out[IDX(i + 1, j + 1, M2)] = g[i + (size_t)M * j].re * inv - shift;
    qgo_fill_ghosts(out, M2, P + 2);
    free(g);
    return 0;
}

/* evolve_psi! (model.jl:172-199) */
void qgo_evolve_psi(const qgo_params *m, const double *zeta, double *psi) {
    const long M2 = m->M + 2, P2 = m->P + 2;
    const size_t F = (size_t)M2 * P2;
    const double a = S1_plus(m), b = S2_minus(m), c = 1 / (a + b);
    const double pi11 = c * b, pi12 = c * a, pi21 = c * -b, pi22 = c * b;
    double *zt1 = malloc(sizeof(double) * F), *zt2 = malloc(sizeof(double) * F);
    double *x1 = malloc(sizeof(double) * F), *x2 = malloc(sizeof(double) * F), *np = malloc(sizeof(double) * F);
    for (size_t q = 0; q < F; ++q) {
        zt1[q] = pi11 * zeta[q] + pi12 * zeta[F + q];
        zt2[q] = pi21 * zeta[q] + pi22 * zeta[F + q];
    }
    qgo_solve(m->M, m->P, m->dx, 0.0, 1, zt1, x1);
    qgo_solve(m->M, m->P, m->dx, S_eig(m), 0, zt2, x2);
    for (int l = 0; l < 2; ++l) {
        for (size_t q = 0; q < F; ++q) np[q] = m->Pfwd[2 * l] * x1[q] + m->Pfwd[2 * l + 1] * x2[q];
        shift3(psi, l, F, np);
    }
    free(zt1); free(zt2); free(x1); free(x2); free(np);
}

/* run_model_no_output.jl:3-16 from the seeded ICs; outputs (M+2,P+2,2,3) each */
int qgo_run(const qgo_params *m, uint64_t seed1, uint64_t seed2, long first_step, long nsteps, double *zeta,
            double *psi, double *f_store, int init, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    const size_t F = (size_t)(m->M + 2) * (m->P + 2);
    if (init) {
        qgo_initialise(m, seed1, seed2, zeta, psi);
        memset(f_store, 0, sizeof(double) * F * 6);
    }
    for (long t = first_step; t < first_step + nsteps; ++t) {
        qgo_evolve_zeta(m, zeta, psi, t, f_store);
        qgo_evolve_psi(m, zeta, psi);
    }
    return 0;
}

int qgo_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
