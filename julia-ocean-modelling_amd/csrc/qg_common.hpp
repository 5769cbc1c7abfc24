// Shared helpers for the gfx950 QG kernels and the C-ABI implementation.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>

#include "qg_mi355.h"

#define QG_HIP(call)                                                                   \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "qg_mi355: %s failed: %s (%s:%d)\n", #call,           \
                         hipGetErrorString(e_), __FILE__, __LINE__);                   \
            return QG_ERR_HIP;                                                         \
        }                                                                              \
    } while (0)

#define QG_CHECK(expr)                                                                 \
    do {                                                                               \
        int s_ = (expr);                                                               \
        if (s_ != QG_OK) return s_;                                                    \
    } while (0)

#define QG_LAUNCH_CHECK() QG_HIP(hipGetLastError())

namespace qg {

constexpr int WAVE = 64;

// Bounded host wait on a stream (ev == nullptr) or an event, for a context with a transport
// attached (comm != nullptr; qg_comm.hip): fails with QG_ERR_RCCL on an RCCL async error or
// when no halo exchange completes within the transport's timeout.  comm == nullptr: a plain
// hipStreamSynchronize / hipEventSynchronize.
int comm_wait(void *comm, hipStream_t s, hipEvent_t ev, const char *what);
// qg_set_form's value for `which` (QG_FORM_*; 0 = the automatic choice)
int form(int which);
int comm_set_timeout(void *comm, double seconds);

__host__ __device__ inline size_t fidx(int64_t i, int64_t j, int64_t ld) {
    return static_cast<size_t>(i) + static_cast<size_t>(ld) * static_cast<size_t>(j);
}

// complex helpers on double2 (x = re, y = im)
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cscale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
// the same on float2 (the F32-arithmetic transforms of the F32 wide-row solver)
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// component type of a complex vector type
template <class C>
struct CxReal;
template <>
struct CxReal<double2> {
    using R = double;
};
template <>
struct CxReal<float2> {
    using R = float;
};
template <class C>
__device__ __forceinline__ C cmake(typename CxReal<C>::R x, typename CxReal<C>::R y) {
    C c;
    c.x = x;
    c.y = y;
    return c;
}
// conversions between the storage / arithmetic complex types
__device__ __forceinline__ void cconv(double2 &d, double2 s) { d = s; }
__device__ __forceinline__ void cconv(float2 &d, double2 s) { d = make_float2((float)s.x, (float)s.y); }
__device__ __forceinline__ void cconv(double2 &d, float2 s) { d = make_double2(s.x, s.y); }
__device__ __forceinline__ void cconv(float2 &d, float2 s) { d = s; }

// Streaming accesses (read or written once per step; non-temporal variants measured no gain).
template <class T>
__device__ __forceinline__ void st_stream(T *p, T v) {
    *p = v;
}
template <class T>
__device__ __forceinline__ T ld_stream(const T *p) {
    return *p;
}

// Write v at interior (i, j) and at every ghost cell that is a periodic image of it
// (edges and the diagonal corners of update_doubly_periodic_bc!).  ghost_rows = 0 skips the
// images in rows -1 / P (multi-GPU slabs get those rows from their neighbours).
template <class T>
__device__ __forceinline__ void store_with_ghosts(T *out, int64_t ld, int64_t M, int64_t P,
                                                  int64_t i, int64_t j, T v, bool ghost_rows) {
    const int64_t mi = i + 1, mj = j + 1;
    out[fidx(mi, mj, ld)] = v;
    const bool lo_i = (i == 0), hi_i = (i == M - 1);
    if (hi_i) out[fidx(0, mj, ld)] = v;
    if (lo_i) out[fidx(M + 1, mj, ld)] = v;
    if (ghost_rows) {
        const bool lo_j = (j == 0), hi_j = (j == P - 1);
        if (hi_j) out[fidx(mi, 0, ld)] = v;
        if (lo_j) out[fidx(mi, P + 1, ld)] = v;
        if (hi_i && hi_j) out[fidx(0, 0, ld)] = v;
        if (hi_i && lo_j) out[fidx(0, P + 1, ld)] = v;
        if (lo_i && lo_j) out[fidx(M + 1, P + 1, ld)] = v;
        if (lo_i && hi_j) out[fidx(M + 1, 0, ld)] = v;
    }
}

// Same as store_with_ghosts for a whole row j that the caller walks: `row` = out + (j+1)*ld
// and the ghost-row target `grow` (row 0 when j == P-1, row P+1 when j == 0, else nullptr)
// are wave-uniform, so every store is an SGPR base + 32-bit lane offset.
// EDGE = false: i is neither column 0 nor M-1 (a strip away from the row ends)
template <class T, bool EDGE = true>
__device__ __forceinline__ void store_row_with_ghosts(T *row, T *grow, int M, int i, T v) {
    st_stream(row + i + 1, v);
    if constexpr (!EDGE) {
        if (grow) grow[i + 1] = v;
        return;
    }
    if (i == M - 1) row[0] = v;
    if (i == 0) row[M + 1] = v;
    if (grow) {
        grow[i + 1] = v;
        if (i == M - 1) grow[0] = v;
        if (i == 0) grow[M + 1] = v;
    }
}

template <class T>
__device__ __forceinline__ T *ghost_row_target(T *out, int64_t ld, int64_t P, int64_t j, bool ghost_rows) {
    if (!ghost_rows) return nullptr;
    if (j == P - 1) return out;                                     // ghost row j = -1
    if (j == 0) return out + static_cast<size_t>(P + 1) * ld;       // ghost row j = P
    return nullptr;
}

// XCD-aware workgroup order.  The dispatcher deals workgroups round-robin to the 8 XCDs
// (linear id b -> XCD b % 8), each XCD with its own L2; this maps b to a logical id such that
// each XCD receives a contiguous range of logical ids (the remainder W mod 8 keeps its id), so
// workgroups that share data (neighbouring strips, the two systems of a wide-row chunk) share
// an L2 and run at about the same time.
constexpr int NUM_XCD = 8;
__device__ __forceinline__ int xcd_logical_id() {
    const int W = gridDim.x * gridDim.y * gridDim.z;
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int full = W - W % NUM_XCD;
    return b < full ? (b % NUM_XCD) * (full / NUM_XCD) + b / NUM_XCD : b;
}

// counter-based uniform in [0,1) shared with oracle/qg_ref.py and oracle/qg_oracle.c
__host__ __device__ inline double u01(uint64_t seed, uint64_t k) {
    uint64_t x = seed + (k + 1) * 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    x = x ^ (x >> 31);
    return static_cast<double>(x >> 11) * 0x1.0p-53;
}

// Model-derived constants, in the reference's evaluation order (src/model.jl:109-121).
struct Derived {
    double ratio, S1, S2, beta1, beta2, Seig;
    double Pinv[4];  // P_inv_matrix (model.jl:90-99), row-major
};

inline Derived derive(const qg_params &m) {
    Derived d;
    d.ratio = 0.5 * (m.H_1 + m.H_2) / ((m.R_d * m.R_d) * ((1 / m.H_1) + (1 / m.H_2)));
    d.S1 = (2 * d.ratio) / (m.H_1 * (m.H_1 + m.H_2));
    d.S2 = (2 * d.ratio) / (m.H_2 * (m.H_1 + m.H_2));
    d.beta1 = m.beta + (d.S1 * m.U);
    d.beta2 = m.beta - (d.S2 * m.U);
    d.Seig = -1 / (m.R_d * m.R_d);
    const double a = d.S1, b = d.S2, c = 1 / (a + b);
    d.Pinv[0] = c * b;
    d.Pinv[1] = c * a;
    d.Pinv[2] = c * -b;
    d.Pinv[3] = c * b;
    return d;
}

// ---- stencil / tendency launchers (qg_stencil.hip) ----------------------------------
// T = element type of the state fields (double: the reference's Float64; float: the F32
// build of BASELINE config 5)
template <class T>
struct RowSrcT {
    // Rows outside [0, P) of a field come from these pointers (interior element 0 of the
    // row, i.e. already offset by the left ghost): index 0,1 = rows -2,-1; 2,3 = rows P, P+1.
    const T *halo[4];
};
using RowSrc = RowSrcT<double>;

template <class T>
struct TendArgsT {
    int64_t M, P, ld;          // interior sizes; ld = M + 2
    double dx, visc, dt, U, r;
    double beta[2];
    int ab3;                   // 0 = Euler, 1 = AB3
    int j0, j1;                // output row range [j0, j1)
    int j2, j3;                // optional second range [j2, j3) (empty: j3 <= j2)
    int write_ghost_rows;      // single-GPU: refresh ghost rows -1 and P
    // per layer pointers (field base = element (0,0) incl. ghosts)
    const T *zeta[2];
    const T *psi[2];
    const T *fprev1[2];   // F(t-1), F(t-2) for AB3
    const T *fprev2[2];
    T *zeta_out[2];
    T *f_out[2];
    // store_new_state!'s shift of f_store fused into the AB3 step (keep-order drop-in, one
    // rank): F(t-1) -> fshift1, F(t-2) -> fshift2 with their ghost images, point by point
    // after they are read (fprev1 / fprev2 are then slots 1 / 2, f_out slot 1); nullptr: off
    T *fshift1[2];
    T *fshift2[2];
    RowSrcT<T> zeta_rows[2];
    RowSrcT<T> psi_rows[2];
    const double *wind;        // [P] upper-layer wind forcing per local row, or nullptr (off)
    // PCG certification fused into the next tendency (launch_tendency_cert, F64, one rank):
    // per workgroup (b,b), (r,r) of both systems for the solve that produced psi from zeta
    double *cert;              // [workgroups][4] partials
    double cert_in[4];         // proj_in (b_s = -(proj_in zeta)_s)
    double cert_pinv[4];       // P_fwd^-1 (psi~ = P_fwd^-1 psi)
    double cert_alpha[2];      // construct_spA shifts
    int cert_pin;              // system 0 pinned at interior (0, 0)
};
using TendArgs = TendArgsT<double>;

// double-gyre wind forcing of local row j of a slab at global row offset j0 (qg_params)
inline double wind_row(double tau0, double rho0, double H1, double dx, int64_t P_total, int64_t jg) {
    const double pi2 = 6.283185307179586;
    const double A = (pi2 * tau0) / (rho0 * H1 * ((double)P_total * dx));
    return -A * std::sin(pi2 * (((double)jg + 0.5) / (double)P_total));
}

int launch_tendency(const TendArgsT<double> &a, hipStream_t s);
int launch_tendency(const TendArgsT<float> &a, hipStream_t s);
// the same tendency, both layers per workgroup, also certifying the previous solve (a.cert):
// *nblk = workgroups launched (partials written); a grid of more than `cap` workgroups (the
// partials' capacity) is refused before anything is launched
int launch_tendency_cert(const TendArgsT<double> &a, int64_t cap, int *nblk, hipStream_t s);
int launch_laplace(const double *u, double *out, int64_t M, int64_t P, double dx, hipStream_t s);
int launch_cd(const double *u, double *out, int64_t M, int64_t P, double dx, hipStream_t s);
int launch_arakawa(const double *z, const double *p, double *out, int64_t M, int64_t P, double dx,
                   hipStream_t s);
int launch_fill_ghosts(double *b, int64_t M, int64_t P, hipStream_t s);
int launch_fill_ghost_cols(double *b, int64_t M, int64_t P, hipStream_t s);
// in-place slot moves of (M+2, P+2, 2, 3) arrays: new slot q <- old slot src[k][q] (-1: kept)
// (slot_bytes = bytes of one slot, both layers; a multiple of 16)
int launch_slot_move(void *const *arrays, const int (*src)[3], int narrays, size_t slot_bytes, hipStream_t s);
// store_new_state!'s shift (slot 3 <- slot 2 <- slot 1) of n arrays
inline int launch_slot_shift(void *const *arrays, int narrays, size_t slot_bytes, hipStream_t s) {
    static const int sh[3][3] = {{-1, 0, 1}, {-1, 0, 1}, {-1, 0, 1}};
    return launch_slot_move(arrays, sh, narrays, slot_bytes, s);
}
// esize = sizeof(element) of the state fields (8 or 4)
int launch_initialise_global(void *zeta, void *psi, void *f_store, int esize, int64_t M, int64_t P,
                             int64_t P_total, int64_t j_offset, double amp, double S1, double S2,
                             double dx, uint64_t seed1, uint64_t seed2, hipStream_t s);

}  // namespace qg
