// Direct periodic 5-point solver for the pair of systems of evolve_psi! (Poisson, pinned;
// modified Helmholtz), replacing the two CHOLMOD factors (src/schemes/laplacian.jl:60-75,
// solves at src/model.jl:186,191).
//
// Method (FACR(0): Fourier in x, tridiagonal in y):
//   1. pass A   one workgroup per chunk of L rows.  Each row of the two right-hand sides is
//               projected, packed as z = f1 + i f2, DFT'd in LDS, split into the two
//               half-spectra; every wavenumber k then runs the backward first-order filter
//               u_j = cs_k F_j + r_k u_{j+1} of the cyclic tridiagonal line solve
//               X_{j-1} - 2 rho_k X_j + X_{j+1} = dx^2 F_j (factored as (1-rS)(1-rS^-1); the
//               output scale cs_k = -r_k dx^2 / M is applied up front, everything after is
//               linear), chunk-local (zero carry).  Writes u (the only full-size
//               intermediate) and two complex chunk summaries per (system, k).
//   2. carry    segment-parallel scans over chunks -> chunk carry-ins (local to this rank)
//               and rank aggregates.
//   3. [RCCL all-gather of the rank records when the y direction is split over GPUs]
//   4. pin      one workgroup: cross-rank carries, Poisson compatibility shift delta, the
//               singular k = 0 Poisson line (double prefix sum), the pinning value.
//   5. pass B   one workgroup per chunk: forward filter X_j = u_true_j + r X_{j-1} with the
//               carries, inverse DFT in LDS, pin, back-projection, store with the ghost ring.
// HBM traffic per grid point for both systems: read 2 + write 2 (pass A), read 2 + write 2
// (pass B) doubles, plus ~0.5 double of chunk summaries.
// Wide rows (M = 8192): the per-wavenumber recurrence state of both systems does not fit in a
// CU's registers next to the transform, so passes A and B run one system per workgroup, each
// real row transformed as a half-length (M/2) complex FFT plus a split step; pass A reads
// both inputs once per system, pass B hands system 0's rows to the system-1 launch through
// half_tmp: 12 instead of 8 doubles per point, without register spills.
#pragma once

#include "qg_common.hpp"

namespace qg {

struct Coef {  // per (system, k); see SpectralSolver::init
    double r, rinv, lr, q, gam, rP, gamP, cs, inv1mrPt, qm1;  // qm1 = r^(L-1)
};

struct SpecArgs {
    int64_t M, P, ld;         // M = row length (2^k, or even <= 2048), P = local rows, ld = M + 2
    int64_t P_total;          // global rows
    int rank, nranks;
    int L, Nc, KH, KS;        // chunk rows, chunks, M/2+1, padded k stride
    double dx;
    int pinned0;              // system 0 is the pinned Poisson problem
    double pin_in[4];         // projection of the inputs
    double pin_out[4];        // back-projection of the outputs
    int write_ghost_rows;
    int f32;                  // the fields are float (F32 state), else double
    const void *in1, *in2;    // (M+2, P+2) fields
    void *out1, *out2;
    const double2 *tw;        // M twiddles
    const Coef *coef;         // [2][KS]
    const double2 *crr;       // [2][KS] (r, 1/r) of coef, unit-stride for the row loops
    const double *ccs;        // [2][KS] cs of coef
    const double *cr;         // [2][KS] r of coef: pass A's one 8-byte load per line and row
    double csc;               // -dx^2 / M: cs = r csc (pass A forms cs on the fly)
    // M = 4096 / 8192 (the lane-exchange passes): r and (r, 1/r) in SLOT order, [2][KS] with
    // slot t + 512 q holding thread t's line q (qg_fft_lx.hpp's mirror groups); the passes also
    // keep u in slot order (U is private to them), so every row access is one aligned run per
    // wave.  Slot 0 of thread 0 is the line k = 0 (u packs k = 0 and k = M/2 there).
    const double *scr;
    const double2 *scrr;
    void *U;                  // [P][2][KS] complex (double2, or float2 for F32 states); k order,
                              // slot order in the lane-exchange passes
    double2 *ULS, *WLS;       // [Nc][2][KS]
    double2 *UIN, *WIN;       // [Nc][2][KS]
    double *dcpart;           // [Nc]
    double *rec;              // this rank's record (see rec_* offsets)
    const double *grec;       // gathered records [nranks] (== rec when nranks == 1)
    int64_t rec_stride;       // doubles per record
    double2 *EXT;             // [2 (Uext, Wext)][2][KS]
    double *hline;            // [P] k = 0 Poisson line h_j of this rank (pass A)
    double *line;             // [P] centred local part of the singular line, scaled (carry)
    double *scal;             // [0] = delta, [1] = pin, [2] [3]: singular-line offset, slope
    double *pinpart;          // per-workgroup parts of the pin value (spec_pin -> pass B)
    const double2 *tw2;       // wide rows (M = 8192): M/2 twiddles of the half-length FFT
    void *half_tmp;           // wide rows: [P][M] system-0 result, state precision (pass B 0 -> 1)
    int nrad, rad[16];        // generic rows: mixed-radix pass plan (0 = direct DFT)
    const int *perm;          // split rows with a plan: position of frequency k after the DIF stages
    int fuse_pin;             // one rank: spec_carry also does spec_pin's work
    // rows no transform above takes (odd M > 8192, M > 16384): Bluestein's chirp-z DFT through
    // power-of-two FFTs of length bl_L >= 2M - 1 in global memory, rows in batches of bl_rows
    const double2 *bl_chirp;  // [M] exp(-pi i n^2 / M)
    const double2 *bl_bhat;   // [bl_L] FFT of the filter b_m = exp(+pi i m^2 / M) (m = -(M-1)..M-1), / bl_L
    const double2 *bl_tw;     // [bl_L] exp(-2 pi i m / bl_L)
    double2 *bl_buf0, *bl_buf1;  // [bl_rows][bl_L] ping-pong
    int bl_L, bl_rows;        // bl_L = 0: not a Bluestein row
    // (M+2, P+2) fields, or null: pass A also writes its two inputs there, ghost ring included
    // (single GPU) -- the drop-in lean mode's move of the new zeta into slot 1 (qg_capi.hip)
    void *zcopy1, *zcopy2;
    int npin;                 // pin parts pass B sums (pinpart[0 .. npin))
    // two-point domains (global M = 2 or P = 2, one rank): see spec_twopoint
    int two;                  // 1: this solver is the two-point path
    int two_yline;            // 1: the line runs along y (M = 2, P >= 3), else along x (P = 2)
    int64_t two_N;            // line length
    double two_r[2][2];       // [system][mode] filter root r (N >= 3) or diagonal a (N = 2)
    double two_inv1mrN[2][2]; // 1 / (1 - r^N)
    double *two_X;            // [2][2][N] line solutions
    double *two_z;            // [N][2] A0^-1 e_1 of the unpinned Poisson operator (the pin)
};

// record layout (doubles)
__host__ __device__ inline int64_t rec_AU(int KS) { return 0; }                 // [2][KS] double2
__host__ __device__ inline int64_t rec_AW(int KS) { return 4 * (int64_t)KS; }  // [2][KS] double2
__host__ __device__ inline int64_t rec_ULS0(int KS) { return 8 * (int64_t)KS; }  // [KS] double2 (sys 0)
__host__ __device__ inline int64_t rec_UIN0(int KS) { return 10 * (int64_t)KS; } // [KS] double2 (sys 0)
// [0] sum of the k = 0 Poisson line (-> delta), [1] H = its local total, [2] Q = sum of its
// local prefix sums (the singular line's cross-rank affine correction), [3] unused
__host__ __device__ inline int64_t rec_DSUM(int KS) { return 12 * (int64_t)KS; }
__host__ __device__ inline int64_t rec_size(int KS, int64_t P) { (void)P; return 12 * (int64_t)KS + 4; }

class SpectralSolver {
public:
    // alpha[s]: construct_spA shift; pinned0: system 0 is the pinned Poisson problem
    int init(int64_t M, int64_t P, int64_t P_total, int rank, int nranks, double dx, const double alpha[2],
             int pinned0, const double pin_in[4], const double pin_out[4], int chunk_rows, int f32 = 0);
    ~SpectralSolver();
    static bool supports(int64_t M, int64_t P);
    // enqueue the whole solve; `gather` (may be null) all-gathers rec -> grec across ranks
    typedef int (*GatherFn)(void *user, const double *send, double *recv, int64_t count, hipStream_t s);
    int solve(const void *in1, const void *in2, void *out1, void *out2, int write_ghost_rows,
              hipStream_t s, GatherFn gather = nullptr, void *user = nullptr, const double *pin_in = nullptr,
              const double *pin_out = nullptr,  // optional per-call projections
              void *zcopy1 = nullptr, void *zcopy2 = nullptr);  // see SpecArgs::zcopy1
    // pass A can write the zcopy fields (power-of-two rows: the FFT and wide-row passes)
    bool fuses_input_copy() const { return !a_.two && a_.M >= 8 && a_.M <= 8192 && (a_.M & (a_.M - 1)) == 0; }
    const SpecArgs &args() const { return a_; }
    size_t device_bytes() const { return bytes_; }
    double *gather_buf() const { return grec_buf_; }  // the record all-gather's target

private:
    int init_twopoint(int64_t M, int64_t P, int nranks, double dx, const double alpha[2], int pinned0,
                      const double pin_in[4], const double pin_out[4], int f32);
    SpecArgs a_{};
    void *mem_ = nullptr;
    double *grec_buf_ = nullptr;
    size_t bytes_ = 0;
};

}  // namespace qg
