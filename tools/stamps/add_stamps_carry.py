"""Add wall_clock64 phase stamps to spec_carry in a COPY of csrc (experiment builds only):
python tools/stamps/add_stamps_carry.py DIR.  Read back with tools/stamps/stamps_carry.py.
Per workgroup (linear id x + y * gridDim.x) 8 slots: 0 entry, 1 summaries arrived (first use),
2 segment combine done, 3 backward pass (UIN stores issued), 4 forward pass (WIN stores issued),
5 closure (fuse_pin) done, 6 exit after the stores drained (k-block 0 of a packed grid: after the
extra column's work); extra-column workgroups (unpacked grids): 0 and 6."""
import sys

p = sys.argv[1] + '/qg_spectral.hip'
s = open(p).read()
a0 = '''namespace qg {

constexpr int CARRY_WAVES = 8;'''
assert s.count(a0) == 1
s = s.replace(a0, '''namespace qg {
__device__ unsigned long long g_stamp[1024 * 8];
#define STAMP(slot) do { const unsigned _b = blockIdx.x + blockIdx.y * gridDim.x; if (threadIdx.x == 0 && _b < 1024) { unsigned long long _t = wall_clock64(); __builtin_nontemporal_store(_t, &g_stamp[_b * 8 + (slot)]); } } while (0)

constexpr int CARRY_WAVES = 8;''')
i0 = s.index('__global__ __launch_bounds__(64 * CARRY_WAVES, MINW) void spec_carry(SpecArgs a) {')
i1 = s.index('// pin: cross-rank / periodic carries')
seg = s[i0:i1]
body = [
    ("""    constexpr int NT = 64 * CARRY_WAVES;
    const bool pk = a.carry_pack != 0;""", """    constexpr int NT = 64 * CARRY_WAVES;
    STAMP(0);
    const bool pk = a.carry_pack != 0;"""),
    ("""        extra();
        return;
    }""", """        extra();
        __builtin_amdgcn_s_waitcnt(0);
        STAMP(6);
        return;
    }"""),
    ("""    double2 v = make_double2(0, 0);
    double2 qlen = make_double2(1, 1);""", """    asm volatile("" ::"v"(uls[0].x), "v"(wls[CARRY_REG - 1].y));
    STAMP(1);
    double2 v = make_double2(0, 0);
    double2 qlen = make_double2(1, 1);"""),
    ("""        if (g > seg) vin = cfma2(qlen_s[g][kk], vin, agg[g][kk]);
    __syncthreads();
""", """        if (g > seg) vin = cfma2(qlen_s[g][kk], vin, agg[g][kk]);
    __syncthreads();
    STAMP(2);
"""),
    ("""    agg[seg][kk] = bsum;""", """    STAMP(3);
    agg[seg][kk] = bsum;"""),
    ("""    if (seg == CARRY_SEG - 1 && ok) put_rec(a.rec + rec_AW(KS), s * KS, w);""", """    if (seg == CARRY_SEG - 1 && ok) put_rec(a.rec + rec_AW(KS), s * KS, w);
    STAMP(4);"""),
    ("""    if (pk && blockIdx.x == 0) extra();  // (packed grids: no extra column)
}""", """    STAMP(5);
    if (pk && blockIdx.x == 0) extra();  // (packed grids: no extra column)
    __builtin_amdgcn_s_waitcnt(0);
    STAMP(6);
}"""),
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
