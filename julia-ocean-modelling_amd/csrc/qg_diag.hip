// Monitoring diagnostics of the newest state (qg_diagnostics, include/qg_mi355.h):
// update_max / update_min of run_model.jl:41-53 over zeta and psi, circulation, enstrophy,
// kinetic energy and the interface term.  Two launches: per-block partial records over row
// strips, then one block that folds them in a fixed order (deterministic for a given grid).
// Everything accumulates in F64, also for an F32 state.  HBM-bound: 4 fields read once.
#include <cfloat>

#include "qg_common.hpp"

namespace qg {

namespace {

constexpr int DIAG_T = 256;
constexpr int DIAG_MAXB = 512;

// record slots (= the qg_diag field order)
enum { ZMAX = 0, ZMIN = 2, PMAX = 4, PMIN = 6, ZSUM = 8, ENS = 10, KE = 12, IFACE = 14, NREC = 16 };

// slot kinds: maxima, minima, sums
__host__ __device__ constexpr bool is_min(int k) { return (k >= ZMIN && k < ZMIN + 2) || (k >= PMIN && k < PMIN + 2); }
__host__ __device__ constexpr bool is_max(int k) { return k < ZSUM && !is_min(k); }

// NaN-propagating max / min: Julia's maximum / minimum return NaN when the matrix holds one
// (fmax / fmin would drop it and report finite extrema for a diverged run)
__host__ __device__ inline double nmax(double a, double b) { return (a != a || b != b) ? a + b : fmax(a, b); }
__host__ __device__ inline double nmin(double a, double b) { return (a != a || b != b) ? a + b : fmin(a, b); }

__device__ inline double wave_max(double v) {
    for (int o = 32; o > 0; o >>= 1) v = nmax(v, __shfl_xor(v, o));
    return v;
}
__device__ inline double wave_min(double v) {
    for (int o = 32; o > 0; o >>= 1) v = nmin(v, __shfl_xor(v, o));
    return v;
}
__device__ inline double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// fold one record per thread (v[NREC]) into the block's record at out[0..NREC)
__device__ void block_fold(double (&v)[NREC], double *out) {
    __shared__ double red[DIAG_T / WAVE][NREC];
    const int lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
#pragma unroll
    for (int k = 0; k < NREC; ++k) {
        double x = v[k];
        if (is_min(k)) x = wave_min(x);
        else if (is_max(k)) x = wave_max(x);
        else x = wave_sum(x);
        if (lane == 0) red[w][k] = x;
    }
    __syncthreads();
    if (threadIdx.x < NREC) {
        const int k = threadIdx.x;
        double x = red[0][k];
        for (int q = 1; q < DIAG_T / WAVE; ++q) {
            const double y = red[q][k];
            if (is_min(k)) x = nmin(x, y);
            else if (is_max(k)) x = nmax(x, y);
            else x += y;
        }
        out[k] = x;
    }
}

__device__ inline void rec_init(double (&v)[NREC]) {
#pragma unroll
    for (int k = 0; k < NREC; ++k) v[k] = 0.0;
    v[ZMAX] = v[ZMAX + 1] = v[PMAX] = v[PMAX + 1] = -DBL_MAX;
    v[ZMIN] = v[ZMIN + 1] = v[PMIN] = v[PMIN + 1] = DBL_MAX;
}

template <class T>
__global__ void __launch_bounds__(DIAG_T) diag_partial_kernel(const T *__restrict__ z0, const T *__restrict__ z1,
                                                              const T *__restrict__ p0, const T *__restrict__ p1,
                                                              int M, int P, int64_t ld, double *part) {
    double v[NREC];
    rec_init(v);
    for (int j = blockIdx.x; j < P; j += gridDim.x) {
        const size_t r = (size_t)(j + 1) * ld, rn = r + ld;  // row j and row j+1 (ghost at j = P-1)
        for (int i = threadIdx.x; i < M; i += DIAG_T) {
            const T *zs[2] = {z0, z1};
            const T *ps[2] = {p0, p1};
            double pc[2];
#pragma unroll
            for (int l = 0; l < 2; ++l) {
                const double z = (double)zs[l][r + i + 1];
                const double p = (double)ps[l][r + i + 1];
                const double px = (double)ps[l][r + i + 2] - p;   // forward differences (i+1 may be
                const double py = (double)ps[l][rn + i + 1] - p;  // the ghost column, j+1 the ghost row)
                v[ZMAX + l] = nmax(v[ZMAX + l], z);
                v[ZMIN + l] = nmin(v[ZMIN + l], z);
                v[PMAX + l] = nmax(v[PMAX + l], p);
                v[PMIN + l] = nmin(v[PMIN + l], p);
                v[ZSUM + l] += z;
                v[ENS + l] += z * z;
                v[KE + l] += px * px + py * py;
                pc[l] = p;
            }
            const double d = pc[0] - pc[1];
            v[IFACE] += d * d;
        }
    }
    block_fold(v, part + (size_t)blockIdx.x * NREC);
}

// folds nb partial records; applies the dx^2 area element and the 1/2 factors
__global__ void __launch_bounds__(DIAG_T) diag_final_kernel(const double *part, int nb, double dx, double *out) {
    double v[NREC];
    rec_init(v);
    for (int b = threadIdx.x; b < nb; b += DIAG_T) {
        const double *q = part + (size_t)b * NREC;
#pragma unroll
        for (int k = 0; k < NREC; ++k) {
            if (is_min(k)) v[k] = nmin(v[k], q[k]);
            else if (is_max(k)) v[k] = nmax(v[k], q[k]);
            else v[k] += q[k];
        }
    }
    __shared__ double rec[NREC];
    block_fold(v, rec);
    __syncthreads();
    if (threadIdx.x < NREC) {
        const int k = threadIdx.x;
        const double a = dx * dx;
        double x = rec[k];
        if (k == ZSUM || k == ZSUM + 1) x *= a;
        else if (k == ENS || k == ENS + 1) x *= 0.5 * a;
        else if (k == KE || k == KE + 1) x *= 0.5;  // sum (dpsi/dx)^2 dx^2 = sum dpsi^2
        else if (k == IFACE) x *= 0.5 * a;
        out[k] = x;
    }
}

}  // namespace

int diag_record_len() { return NREC; }
size_t diag_scratch_doubles() { return (size_t)DIAG_MAXB * NREC + NREC; }

// rec (device, NREC doubles) <- the rank-local record; scratch from diag_scratch_doubles()
int launch_diagnostics(const void *z0, const void *z1, const void *p0, const void *p1, int esize, int64_t M,
                       int64_t P, double dx, double *scratch, double *rec, hipStream_t s) {
    const int nb = (int)(P < DIAG_MAXB ? P : DIAG_MAXB);
    const int64_t ld = M + 2;
    if (esize == (int)sizeof(float))
        diag_partial_kernel<float><<<nb, DIAG_T, 0, s>>>((const float *)z0, (const float *)z1, (const float *)p0,
                                                         (const float *)p1, (int)M, (int)P, ld, scratch);
    else
        diag_partial_kernel<double><<<nb, DIAG_T, 0, s>>>((const double *)z0, (const double *)z1,
                                                          (const double *)p0, (const double *)p1, (int)M, (int)P,
                                                          ld, scratch);
    QG_LAUNCH_CHECK();
    diag_final_kernel<<<1, DIAG_T, 0, s>>>(scratch, nb, dx, rec);
    QG_LAUNCH_CHECK();
    return QG_OK;
}

}  // namespace qg
