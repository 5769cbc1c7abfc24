"""Add wall_clock64 phase stamps to spec_passB (the 4096-point lane-exchange form) in a COPY of
csrc (experiment builds only): python tools/stamps/add_stamps_pb4k.py DIR.  Read back with
tools/stamps/stamps_phases.py.  Per workgroup 256 slots: 0 entry, 1 rows start, then five per
row (row start, prefetched u converted = arrived, recurrence done = coefficients arrived,
transform done, stores + next coefficient loads issued), 255 exit after the stores drained."""
import sys

p = sys.argv[1] + '/qg_spectral.hip'
s = open(p).read()
a0 = '''namespace qg {

constexpr int CARRY_WAVES = 8;'''
assert s.count(a0) == 1
s = s.replace(a0, '''namespace qg {
__device__ unsigned long long g_stamp[1024 * 256];
#define STAMP(slot) do { if (threadIdx.x == 0 && blockIdx.x < 1024) { unsigned long long _t = wall_clock64(); __builtin_nontemporal_store(_t, &g_stamp[blockIdx.x * 256 + (slot)]); } } while (0)

constexpr int CARRY_WAVES = 8;''')
i0 = s.index('__global__ __launch_bounds__(Geo<N>::T, Geo<N>::MINW) void spec_passB(SpecArgs a) {')
i1 = s.index('// Wide rows (M = 8192).  Both systems')
seg = s[i0:i1]
body = [
    ('''    TwFill<N, T> twf;
    if constexpr (!LX) fft_twiddle_load<N, T>(twf, a.tw);''', '''    STAMP(0);
    TwFill<N, T> twf;
    if constexpr (!LX) fft_twiddle_load<N, T>(twf, a.tw);'''),
    ('''    if (blockIdx.x == 0 && t == 0) a.scal[1] = pin;
    for (int j = s0; j <= e; ++j) {
        if constexpr (!PF) load_u(j);''', '''    if (blockIdx.x == 0 && t == 0) a.scal[1] = pin;
    STAMP(1);
    for (int j = s0; j <= e; ++j) {
        const int rs_ = 2 + 5 * (j - s0);
        STAMP(rs_);
        if constexpr (!PF) load_u(j);'''),
    ('''        if (PF && j < e) load_u(j + 1);
        // compiler memory barrier''', '''        asm volatile("" ::"v"(ucur[0][0].x), "v"(ucur[KQ - 1][1].y));
        STAMP(rs_ + 1);
        if (PF && j < e) load_u(j + 1);
        // compiler memory barrier'''),
    ('''        double2 xo[Plan::R_LAST];  // last FFT pass output in registers: element t + r*T
        if constexpr (LX) {''', '''        if constexpr (LX) asm volatile("" ::"v"(zr[0].x), "v"(zm[KQ - 1].y));
        STAMP(rs_ + 2);
        double2 xo[Plan::R_LAST];  // last FFT pass output in registers: element t + r*T
        if constexpr (LX) {'''),
    ('''        S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
        S *row1 = out1 + (size_t)(j + 1) * ld;
        const bool pin_row''', '''        asm volatile("" ::"v"(xo[0].x), "v"(xo[7].y));
        STAMP(rs_ + 3);
        S *out1 = static_cast<S *>(a.out1), *out2 = static_cast<S *>(a.out2);
        S *row1 = out1 + (size_t)(j + 1) * ld;
        const bool pin_row'''),
    ('''        if (j < e) load_coef();
        if constexpr (!LX && Inv::b0_read_late) __syncthreads();  // the next row's recurrence writes b0
    }
#undef QG_PB_R
}''', '''        if (j < e) load_coef();
        STAMP(rs_ + 4);
        if constexpr (!LX && Inv::b0_read_late) __syncthreads();  // the next row's recurrence writes b0
    }
    __builtin_amdgcn_s_waitcnt(0);
    STAMP(255);
#undef QG_PB_R
}'''),
]
for a, b in body:
    assert seg.count(a) == 1, a[:70]
    seg = seg.replace(a, b)
s = s[:i0] + seg + s[i1:]
s += '''
extern "C" int qg_debug_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(qg::g_stamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -3;
}
'''
open(p, 'w').write(s)
