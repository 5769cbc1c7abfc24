// 4096-point complex transform of one row by a workgroup of 512 threads (eight waves), eight
// values per thread, with TWO LDS round trips per row instead of the Stockham plan's four
// (qg_fft.hpp).  The row length and thread count are those of the 4096^2 passes and of the
// wide-row (M = 8192) half-length transforms.
//
// Index digits (radix 8): input n = d0 + 8 d1 + 64 d2 + 512 d3, output k = c0 + 8 c1 + 64 c2
// + 512 c3.  W = exp(-+2 pi i / 4096).  n k mod 4096 splits into
//   d3 c0 512                      -> stage 1: DFT8 over d3, no twiddle
//   d2 (c0 64 + c1 512)            -> stage 2: twiddle W^(64 d2 c0), DFT8 over d2
//   d1 (c0 8 + c1 64 + c2 512)     -> stage 3: twiddle W^(8 d1 (c0 + 8 c1)), DFT8 over d1
//   d0 (c0 + 8 c1 + 64 c2 + 512 c3)-> stage 4: twiddle W^(d0 (c0 + 8 c1 + 64 c2)), DFT8 over d0
// Each stage needs its digit in a thread's eight registers.  Where the other three digits
// sit (lane bits 0-2, lane bits 3-5, wave) is free, and moves between stages are:
//   T1 (LDS, after stage 1): register <-> wave transpose; afterwards wave = c0, lane bits 3-5 =
//      d1, lane bits 0-2 = d0, registers = d2;
//   X  (no LDS, after stage 2): registers <-> lane bits 3-5, a 2x2 transpose per bit --
//      lane bit 5 by v_permlane32_swap, bit 4 by v_permlane16_swap (gfx950; one instruction
//      per dword pair), bit 3 by two DPP row_ror:8 moves with bank masks;
//   T2 (LDS, after stage 3): registers <-> d0, and the thread -> output-group map the caller
//      wants (natural for coalesced row stores, or `mirror_group` for the real-data split).
// The LDS traffic per row is two writes and two reads of the row (the Stockham plan: four
// each, plus the split step's reads), two barriers.
//
// Thread -> group maps.  A thread owns the eight elements g + 512 r (r = register) of its group
// g < 512 at the input of stage 1 (IN_MIRROR: g = mirror_group(t), else g = t) and at the
// output of stage 4 (OUT_MIRROR likewise).  mirror_group puts the group 512 - g in the lane 32
// places up or down of g in the same wave (groups 0 and 256, their own mirrors, sit in lanes 0
// and 32 of wave 0), so element pairs (k, 4096 - k) -- what a real-data split pairs -- are
// exchanged by `mirror_exchange` in registers: k = g + 512 r pairs with 4096 - k = (512 - g) +
// 512 (7 - r), i.e. the partner lane's register 7 - r.
//
// LDS layouts.  T1: element (c0, g) at c0 * 512 + g -- writer and reader instructions touch 64
// consecutive elements (conflict-free ds_write_b128 / ds_read_b128).  T2: element (d0, m) at
// d0 * 512 + (m ^ d0): the writer's 8-lane groups (d0 = 0..7, one m) hit eight distinct 16-B
// slots, the reader's 16 consecutive m stay distinct modulo 16.
//
// Twiddles: `tw512` (LDS, caller-filled) holds W^m, m < 512, of the forward 4096-point table; a
// stage uses one entry as its base w and forms w^r by repeated multiplication (as qg_fft.hpp).
#pragma once

#include "qg_fft.hpp"

namespace qg {
namespace lx {

constexpr int N = 4096, T = 512;
constexpr int LDS_ELEMS = 2 * N + 512 + 8;  // T1 buffer, T2 buffer, tw512, the mirror stash

__host__ __device__ __forceinline__ int mirror_group(int t) {
    const int w = t >> 6, l = t & 63, j = l & 31, g = 32 * w + j;
    return l < 32 ? g : (g == 0 ? 256 : 512 - g);
}

__device__ __forceinline__ unsigned lo32(double x) { return (unsigned)__double2loint(x); }
__device__ __forceinline__ unsigned hi32(double x) { return (unsigned)__double2hiint(x); }
__device__ __forceinline__ double mkd(unsigned lo, unsigned hi) { return __hiloint2double((int)hi, (int)lo); }

// 2x2 transpose (register bit <-> lane bit 5) of the dword pair (a, b): a keeps lanes 0-31 and
// takes b's lanes 0-31 into lanes 32-63; b takes a's lanes 32-63 into lanes 0-31
__device__ __forceinline__ void pl32(unsigned &a, unsigned &b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
// the same for lane bit 4 (rows of 16 lanes)
__device__ __forceinline__ void pl16(unsigned &a, unsigned &b) {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
// the same for lane bit 3: row_ror:8 reaches the lane 8 away within a row of 16; bank_mask
// selects the lanes written (banks 0-1: lane bit 3 = 0, banks 2-3: = 1)
__device__ __forceinline__ void dpp8(unsigned &a, unsigned &b) {
    const int a0 = (int)a, b0 = (int)b;
    a = (unsigned)__builtin_amdgcn_update_dpp(a0, b0, 0x128, 0xf, 0xc, false);
    b = (unsigned)__builtin_amdgcn_update_dpp(b0, a0, 0x128, 0xf, 0x3, false);
}

template <int LB>
__device__ __forceinline__ void xpose(double2 &p, double2 &q) {  // p: register bit 0, q: bit 1
    unsigned a[4] = {lo32(p.x), hi32(p.x), lo32(p.y), hi32(p.y)};
    unsigned b[4] = {lo32(q.x), hi32(q.x), lo32(q.y), hi32(q.y)};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (LB == 5) pl32(a[i], b[i]);
        else if constexpr (LB == 4) pl16(a[i], b[i]);
        else dpp8(a[i], b[i]);
    }
    p = make_double2(mkd(a[0], a[1]), mkd(a[2], a[3]));
    q = make_double2(mkd(b[0], b[1]), mkd(b[2], b[3]));
}

// registers <-> lane bits 3-5 (register bit i <-> lane bit 3 + i)
__device__ __forceinline__ void swap_regs_lanes345(double2 (&v)[8]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) xpose<5>(v[r], v[r + 4]);
#pragma unroll
    for (int r : {0, 1, 4, 5}) xpose<4>(v[r], v[r + 2]);
#pragma unroll
    for (int r : {0, 2, 4, 6}) xpose<3>(v[r], v[r + 1]);
}

// v[4..7] <- the partner lane's v[4..7] (partner: lane +-32), except lanes 0 and 32 of wave 0
// (groups 0 and 256 in the mirror map), which keep their own (`stash`: 8 LDS elements)
__device__ __forceinline__ void mirror_exchange(double2 (&v)[8], double2 *stash, int t) {
    const bool self = (t & ~32) == 0;
    if (self) {
#pragma unroll
        for (int i = 0; i < 4; ++i) stash[(t >> 5) * 4 + i] = v[4 + i];
    }
#pragma unroll
    for (int r = 4; r < 8; r += 2) {
        unsigned a[4] = {lo32(v[r].x), hi32(v[r].x), lo32(v[r].y), hi32(v[r].y)};
        unsigned b[4] = {lo32(v[r + 1].x), hi32(v[r + 1].x), lo32(v[r + 1].y), hi32(v[r + 1].y)};
        // (a, b) -> a: [own a | partner b], b: [partner a | own b]; then (b, a) -> b: partner
        // a everywhere, a: partner b everywhere
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            pl32(a[i], b[i]);
            pl32(b[i], a[i]);
        }
        v[r] = make_double2(mkd(b[0], b[1]), mkd(b[2], b[3]));
        v[r + 1] = make_double2(mkd(a[0], a[1]), mkd(a[2], a[3]));
    }
    if (self) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[4 + i] = stash[(t >> 5) * 4 + i];
    }
}

// twiddle the eight values by w^r (w conjugated for the inverse), then the radix-8 DFT
template <bool INV>
__device__ __forceinline__ void stage(double2 (&v)[8], double2 w) {
    if (INV) w.y = -w.y;
    double2 wr = w;
#pragma unroll
    for (int r = 1; r < 8; ++r) {
        v[r] = cmul(v[r], wr);
        if (r < 7) wr = cmul(wr, w);
    }
    dft8<INV>(v);
}

__device__ __forceinline__ int t2_slot(int d0, int m) { return d0 * 512 + (m ^ d0); }

struct NoHook {
    __device__ void operator()() const {}
};

// Stage 2's twiddle base W^(64 c0) depends on the wave only (c0 = wave), so its powers w^1..w^7
// can be formed once per kernel and held in scalar registers: the row loop then skips the six
// complex multiplies per thread that form them (the same recurrence, so bit-identical values).
struct Stage2Tw {
    double2 p[7];
};
struct NoTw2 {};
__device__ __forceinline__ double uniform_d(double x) {
    return mkd((unsigned)__builtin_amdgcn_readfirstlane((int)lo32(x)),
               (unsigned)__builtin_amdgcn_readfirstlane((int)hi32(x)));
}
template <bool INV>
__device__ __forceinline__ Stage2Tw stage2_powers(const double2 *tw512, int t) {
    double2 w = tw512[64 * (t >> 6)];
    if (INV) w.y = -w.y;
    Stage2Tw s;
    double2 wr = w;
#pragma unroll
    for (int r = 0; r < 7; ++r) {
        s.p[r] = make_double2(uniform_d(wr.x), uniform_d(wr.y));
        if (r < 6) wr = cmul(wr, w);
    }
    return s;
}

// The transform.  v: in: element g_in + 512 r (register r); out: element g_out + 512 r.
// b0, b1: two LDS row buffers (N double2 each); tw512: the LDS twiddle table.  The caller
// guarantees that no thread still reads b0 / b1 from an earlier use when it enters (two calls
// in a row are safe: b0's reads end before T2's barrier, b1's before the next call's T1
// barrier).  `hook` runs after T1's LDS writes, while v holds nothing live (the place for the
// next row's prefetch loads: their registers are not live beside v's).
// ONE_BUF: T2 reuses b0 (b1 is ignored): half the LDS (two workgroups per CU) for two more
// barriers -- T2's writes wait for every wave's T1 reads, and T1's writes for the previous
// call's T2 reads, so the caller needs no guarantee.
// s2: stage 2's twiddle powers (stage2_powers<INV>), or NoTw2 to form them from tw512.
template <bool INV, bool IN_MIRROR, bool OUT_MIRROR, bool ONE_BUF = false, class Hook = NoHook, class Tw2 = NoTw2>
__device__ __forceinline__ void fft(double2 (&v)[8], double2 *b0, double2 *b1, const double2 *tw512, int t,
                                    Hook &&hook = Hook(), const Tw2 &s2 = Tw2()) {
    const int w = t >> 6, l = t & 63;
    if constexpr (ONE_BUF) b1 = b0;
    dft8<INV>(v);  // stage 1 -> c0 in the register index
    if constexpr (ONE_BUF) __syncthreads();
    {
        const int g = IN_MIRROR ? mirror_group(t) : t;
#pragma unroll
        for (int r = 0; r < 8; ++r) b0[r * 512 + g] = v[r];
    }
    hook();
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = b0[w * 512 + r * 64 + l];  // wave c0, register d2
    if constexpr (std::is_same<Tw2, Stage2Tw>::value) {  // -> c1
#pragma unroll
        for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], s2.p[r - 1]);
        dft8<INV>(v);
    } else {
        stage<INV>(v, tw512[64 * w]);
    }
    swap_regs_lanes345(v);             // register d1, lane bits 3-5 c1
    stage<INV>(v, tw512[8 * (w + 8 * (l >> 3))]);  // -> c2
    if constexpr (ONE_BUF) __syncthreads();
    {
        const int d0 = l & 7, mb = w + 8 * (l >> 3);
#pragma unroll
        for (int r = 0; r < 8; ++r) b1[t2_slot(d0, mb + 64 * r)] = v[r];
    }
    __syncthreads();
    const int m = OUT_MIRROR ? mirror_group(t) : t;
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = b1[t2_slot(r, m)];  // register d0
    stage<INV>(v, tw512[m]);           // -> c3
}

// Fill tw512 (caller synchronises): W^m for m < 512 from the forward 4096-point table
__device__ __forceinline__ void fill_tw512(double2 *tw512, const double2 *__restrict__ tw4096) {
    for (int m = threadIdx.x; m < 512; m += blockDim.x) tw512[m] = tw4096[m];
}

}  // namespace lx
}  // namespace qg
