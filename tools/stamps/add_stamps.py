"""Add wall_clock64 phase stamps to spec_passB in a COPY of csrc (experiment builds only):
python tools/stamps/add_stamps.py DIR.  Read back with tools/stamps/stamps_passB.py."""
import sys

p = sys.argv[1] + '/qg_spectral.hip'
s = open(p).read()
rep = [
    ('''namespace qg {

constexpr int CARRY_WAVES = 8;''', '''namespace qg {
__device__ unsigned long long g_stamp[1024 * 64];
#define STAMP(slot) do { if (threadIdx.x == 0 && blockIdx.x < 1024) { unsigned long long _t = wall_clock64(); __builtin_nontemporal_store(_t, &g_stamp[blockIdx.x * 64 + (slot)]); } } while (0)

constexpr int CARRY_WAVES = 8;'''),
    ('''    TwFill<N, T> twf;
    fft_twiddle_load<N, T>(twf, a.tw);
    const int t = threadIdx.x, c = blockIdx.x;
    const int L = a.L, s0 = c * L, e = s0 + L - 1;''', '''    STAMP(0);
    TwFill<N, T> twf;
    fft_twiddle_load<N, T>(twf, a.tw);
    const int t = threadIdx.x, c = blockIdx.x;
    const int L = a.L, s0 = c * L, e = s0 + L - 1;'''),
    ('''    if (blockIdx.x == 0 && t == 0) a.scal[1] = pin;
    for (int j = s0; j <= e; ++j) {''', '''    if (blockIdx.x == 0 && t == 0) a.scal[1] = pin;
    STAMP(1);
    for (int j = s0; j <= e; ++j) {'''),
    ('''        __syncthreads();
        double2 xo[Plan::R_LAST];  // last FFT pass output in registers: element t + r*T
        Inv::run(b0, b1, twl, xo);''', '''        STAMP(2 + 3 * (j - s0));
        __syncthreads();
        double2 xo[Plan::R_LAST];  // last FFT pass output in registers: element t + r*T
        Inv::run(b0, b1, twl, xo);
        STAMP(3 + 3 * (j - s0));'''),
    ('''        if constexpr (Inv::b0_read_late) __syncthreads();  // the next row's recurrence writes b0
    }
#undef QG_PB_R
}''', '''        STAMP(4 + 3 * (j - s0));
        if constexpr (Inv::b0_read_late) __syncthreads();  // the next row's recurrence writes b0
    }
    __builtin_amdgcn_s_waitcnt(0);
    STAMP(63);
#undef QG_PB_R
}'''),
]
a0, b0 = rep[0]
assert s.count(a0) == 1
s = s.replace(a0, b0)
i0 = s.index('void spec_passB(SpecArgs a) {')
i1 = s.index('// Wide rows (M = 8192)')
seg = s[i0:i1]
for a, b in rep[1:]:
    assert seg.count(a) == 1, a[:60]
    seg = seg.replace(a, b)
s = s[:i0] + seg + s[i1:]
s += '''
extern "C" int qg_debug_stamps(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(qg::g_stamp), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -3;
}
'''
open(p, 'w').write(s)
