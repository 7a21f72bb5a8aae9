// MFMA operand hazard probe (not part of the library; DESIGN.md §13e2 and
// round-5 task 4): does v_mfma_f32_32x32x16_{f16,bf16} on gfx950 read a
// SrcB (or SrcA) fragment that a VALU instruction wrote N wait states
// earlier, and does a VALU write N states after the MFMA reach the MFMA
// that is still reading it?
//
// Each wave holds an "old" B fragment, then, inside ONE asm statement (hipcc
// pads nothing inside), rewrites all four B VGPRs by VALU (v_perm_b32 or
// v_mov_b32), issues N s_nop states, and the MFMA.  RAW test: the product
// must use the NEW fragment.  WAR test: the MFMA is issued first, then N
// states, then the VALU rewrite: the product must use the OLD fragment.
// Every lane's 16 results are compared with host-computed references of
// both the old and the new operand (exact small integers in fp16, so the
// fp32 sums are exact); a lane that matches neither, or the wrong one, is
// counted.  Also the compiler's own schedule of the same RAW pattern in plain
// HIP (no asm): `make -C tools hazard` with -save-temps shows its padding.
//
//   hipcc -O3 --offload-arch=gfx950 tools/hazard_probe.hip -o tools/_hazard_probe && tools/_hazard_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef uint32_t frag8 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define NOPS_0 ""
#define NOPS_1 "s_nop 0\n\t"
#define NOPS_2 "s_nop 1\n\t"
#define NOPS_3 "s_nop 2\n\t"
#define NOPS_4 "s_nop 3\n\t"
#define NOPS_8 "s_nop 7\n\t"
#define DRAIN "s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\t"
// B lives in v[200:203], D in v[204:219] (named physical registers, listed
// as clobbers, so hipcc keeps its own values out of them)
#define SET_OLD                                                                                   \
    "v_mov_b32 v200, %[o0]\n\tv_mov_b32 v201, %[o1]\n\tv_mov_b32 v202, %[o2]\n\tv_mov_b32 v203, %[o3]\n\t"
#define PERM_NEW                                                                                  \
    "v_perm_b32 v200, %[h0], %[l0], %[sel]\n\tv_perm_b32 v201, %[h1], %[l1], %[sel]\n\t"   \
    "v_perm_b32 v202, %[h2], %[l2], %[sel]\n\tv_perm_b32 v203, %[h3], %[l3], %[sel]\n\t"
#define MOV_NEW                                                                                   \
    "v_mov_b32 v200, %[l0]\n\tv_mov_b32 v201, %[l1]\n\tv_mov_b32 v202, %[l2]\n\tv_mov_b32 v203, %[l3]\n\t"
#define MFMA "v_mfma_f32_32x32x16_f16 v[204:219], %[a], v[200:203], 0\n\t"
#define MFMA_BF "v_mfma_f32_32x32x16_bf16 v[204:219], %[a], v[200:203], 0\n\t"
#define COPY_OUT                                                                                  \
    "v_mov_b32 %[d0], v204\n\tv_mov_b32 %[d1], v205\n\tv_mov_b32 %[d2], v206\n\tv_mov_b32 %[d3], v207\n\t"     \
    "v_mov_b32 %[d4], v208\n\tv_mov_b32 %[d5], v209\n\tv_mov_b32 %[d6], v210\n\tv_mov_b32 %[d7], v211\n\t"     \
    "v_mov_b32 %[d8], v212\n\tv_mov_b32 %[d9], v213\n\tv_mov_b32 %[d10], v214\n\tv_mov_b32 %[d11], v215\n\t"   \
    "v_mov_b32 %[d12], v216\n\tv_mov_b32 %[d13], v217\n\tv_mov_b32 %[d14], v218\n\tv_mov_b32 %[d15], v219"
#define OUTS                                                                                      \
    [d0] "=&v"(d[0]), [d1] "=&v"(d[1]), [d2] "=&v"(d[2]), [d3] "=&v"(d[3]), [d4] "=&v"(d[4]),      \
    [d5] "=&v"(d[5]), [d6] "=&v"(d[6]), [d7] "=&v"(d[7]), [d8] "=&v"(d[8]), [d9] "=&v"(d[9]),      \
    [d10] "=&v"(d[10]), [d11] "=&v"(d[11]), [d12] "=&v"(d[12]), [d13] "=&v"(d[13]),              \
    [d14] "=&v"(d[14]), [d15] "=&v"(d[15])
#define INS                                                                                       \
    [a] "v"(a), [o0] "v"(bo[0]), [o1] "v"(bo[1]), [o2] "v"(bo[2]), [o3] "v"(bo[3]), [l0] "v"(lo[0]),  \
    [l1] "v"(lo[1]), [l2] "v"(lo[2]), [l3] "v"(lo[3]), [h0] "v"(hi[0]), [h1] "v"(hi[1]),            \
    [h2] "v"(hi[2]), [h3] "v"(hi[3]), [sel] "s"(0x05040100u)
#define CLOB                                                                                      \
    "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", \
    "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219"

#define PROBE_KERNEL(NAME, BODY)                                                                  \
    __global__ __launch_bounds__(512) void NAME(const uint32_t* in, float* out, int iters) {     \
        const int lane = threadIdx.x & 63;                                                        \
        const size_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;                      \
        frag8 a, bo, lo, hi;                                                                      \
        for (int q = 0; q < 4; ++q) {                                                             \
            a[q] = in[lane * 4 + q];                                                              \
            bo[q] = in[256 + lane * 4 + q];                                                       \
            lo[q] = in[512 + lane * 4 + q];                                                       \
            hi[q] = in[768 + lane * 4 + q];                                                       \
        }                                                                                         \
        int nbad = 0;                                                                             \
        float first[16];                                                                          \
        for (int it = 0; it < iters; ++it) {                                                      \
            float d[16];                                                                          \
            asm volatile(BODY COPY_OUT : OUTS : INS : CLOB);                                      \
            if (it == 0)                                                                          \
                for (int r = 0; r < 16; ++r) first[r] = d[r];                                     \
            for (int r = 0; r < 16; ++r) nbad += d[r] != first[r];                                \
        }                                                                                         \
        for (int r = 0; r < 16; ++r) out[(w * 64 + lane) * 16 + r] = first[r];                   \
        out[(size_t)gridDim.x * (blockDim.x / 64) * 64 * 16 + w * 64 + lane] = (float)nbad;      \
    }

// RAW: the VALU rewrite of B, N states, the MFMA (must see the NEW B)
PROBE_KERNEL(raw_perm_0, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_0 MFMA DRAIN)
PROBE_KERNEL(raw_perm_1, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_1 MFMA DRAIN)
PROBE_KERNEL(raw_perm_2, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_2 MFMA DRAIN)
PROBE_KERNEL(raw_perm_3, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_3 MFMA DRAIN)
PROBE_KERNEL(raw_perm_4, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_4 MFMA DRAIN)
PROBE_KERNEL(raw_perm_8, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_8 MFMA DRAIN)
// WAR: the MFMA, N states, the VALU rewrite of B (must see the OLD B)
PROBE_KERNEL(war_mov_0, SET_OLD "s_nop 7\n\t" MFMA NOPS_0 MOV_NEW DRAIN)
PROBE_KERNEL(war_mov_1, SET_OLD "s_nop 7\n\t" MFMA NOPS_1 MOV_NEW DRAIN)
PROBE_KERNEL(war_mov_2, SET_OLD "s_nop 7\n\t" MFMA NOPS_2 MOV_NEW DRAIN)
PROBE_KERNEL(war_mov_4, SET_OLD "s_nop 7\n\t" MFMA NOPS_4 MOV_NEW DRAIN)
PROBE_KERNEL(war_mov_8, SET_OLD "s_nop 7\n\t" MFMA NOPS_8 MOV_NEW DRAIN)

// WAR with the matrix pipe busy: the MFMA that reads B issues behind another
// MFMA (on its own accumulator, or on the same one: a dependent chain), then
// N states, then the VALU rewrite of B.  Q = v[204:219], P = v[220:235]
#define MFMA_P_OTHER "v_mfma_f32_32x32x16_f16 v[220:235], %[a], %[hv], 0\n\t"
#define MFMA_Q_OTHER "v_mfma_f32_32x32x16_f16 v[204:219], %[a], %[hv], 0\n\t"
#define MFMA_Q_DEP "v_mfma_f32_32x32x16_f16 v[204:219], %[a], v[200:203], v[204:219]\n\t"
#define CLOB2 CLOB, "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", \
    "v231", "v232", "v233", "v234", "v235"
#define PROBE_KERNEL2(NAME, BODY)                                                                 \
    __global__ __launch_bounds__(512) void NAME(const uint32_t* in, float* out, int iters) {     \
        const int lane = threadIdx.x & 63;                                                        \
        const size_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;                      \
        frag8 a, bo, lo, hi;                                                                      \
        for (int q = 0; q < 4; ++q) {                                                             \
            a[q] = in[lane * 4 + q];                                                              \
            bo[q] = in[256 + lane * 4 + q];                                                       \
            lo[q] = in[512 + lane * 4 + q];                                                       \
            hi[q] = in[768 + lane * 4 + q];                                                       \
        }                                                                                         \
        int nbad = 0;                                                                             \
        float first[16];                                                                          \
        for (int it = 0; it < iters; ++it) {                                                      \
            float d[16];                                                                          \
            asm volatile(BODY COPY_OUT : OUTS : INS, [hv] "v"(hi) : CLOB2);                       \
            if (it == 0)                                                                          \
                for (int r = 0; r < 16; ++r) first[r] = d[r];                                     \
            for (int r = 0; r < 16; ++r) nbad += d[r] != first[r];                                \
        }                                                                                         \
        for (int r = 0; r < 16; ++r) out[(w * 64 + lane) * 16 + r] = first[r];                   \
        out[(size_t)gridDim.x * (blockDim.x / 64) * 64 * 16 + w * 64 + lane] = (float)nbad;      \
    }
// behind an independent MFMA: Q = A x B_old
PROBE_KERNEL2(war_busy_indep_0, SET_OLD "s_nop 7\n\t" MFMA_P_OTHER MFMA NOPS_0 MOV_NEW DRAIN)
PROBE_KERNEL2(war_busy_indep_2, SET_OLD "s_nop 7\n\t" MFMA_P_OTHER MFMA NOPS_2 MOV_NEW DRAIN)
// dependent chain: Q = A x hi, then Q += A x B_old (must not see B_new)
PROBE_KERNEL2(war_busy_dep_0, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_Q_DEP NOPS_0 MOV_NEW DRAIN)
PROBE_KERNEL2(war_busy_dep_1, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_Q_DEP NOPS_1 MOV_NEW DRAIN)
PROBE_KERNEL2(war_busy_dep_2, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_Q_DEP NOPS_2 MOV_NEW DRAIN)
PROBE_KERNEL2(war_busy_dep_4, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_Q_DEP NOPS_4 MOV_NEW DRAIN)
PROBE_KERNEL2(war_busy_dep_8, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_Q_DEP NOPS_8 MOV_NEW DRAIN)
// RAW behind an independent MFMA: Q = A x B_new
PROBE_KERNEL2(raw_busy_0, SET_OLD "s_nop 7\n\t" MFMA_P_OTHER PERM_NEW NOPS_0 MFMA DRAIN)
PROBE_KERNEL2(raw_busy_1, SET_OLD "s_nop 7\n\t" MFMA_P_OTHER PERM_NEW NOPS_1 MFMA DRAIN)

// The bf16x3 DFT's compiled schedule: two accumulators
// interleaved, so the MFMA that reads B waits behind the other accumulator's
// MFMA AND for its own accumulator from two MFMAs back; the four B registers
// are rewritten by v_perm_b32 right after it, then read (new) by the next
// MFMA.  Q must hold hi + old (or 2 hi + old in the longer chain).
#define MFMA_P_DEP_NEW "v_mfma_f32_32x32x16_f16 v[220:235], %[a], v[200:203], v[220:235]\n\t"
#define MFMA_Q_DEP_HI "v_mfma_f32_32x32x16_f16 v[204:219], %[a], %[hv], v[204:219]\n\t"
#define MFMA_P_DEP_HI "v_mfma_f32_32x32x16_f16 v[220:235], %[a], %[hv], v[220:235]\n\t"
PROBE_KERNEL2(war_inter_perm_0, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_P_OTHER MFMA_Q_DEP NOPS_0 PERM_NEW "s_nop 1\n\t" MFMA_P_DEP_NEW DRAIN)
PROBE_KERNEL2(war_inter_perm_1, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_P_OTHER MFMA_Q_DEP NOPS_1 PERM_NEW "s_nop 1\n\t" MFMA_P_DEP_NEW DRAIN)
PROBE_KERNEL2(war_inter_perm_4, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_P_OTHER MFMA_Q_DEP NOPS_4 PERM_NEW "s_nop 1\n\t" MFMA_P_DEP_NEW DRAIN)
PROBE_KERNEL2(war_inter_chain_0, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_P_OTHER MFMA_Q_DEP_HI MFMA_P_DEP_HI MFMA_Q_DEP NOPS_0 PERM_NEW "s_nop 1\n\t" MFMA_P_DEP_NEW DRAIN)
// RAW into the stalled dependent MFMA at 1 and 2 states (hipcc pads 2)
PROBE_KERNEL2(raw_inter_1, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_P_OTHER PERM_NEW NOPS_1 MFMA_Q_DEP DRAIN)
PROBE_KERNEL2(raw_inter_2, SET_OLD "s_nop 7\n\t" MFMA_Q_OTHER MFMA_P_OTHER PERM_NEW NOPS_2 MFMA_Q_DEP DRAIN)

// WAR on a DS read's ADDRESS register: ds_read_b64 from the address in v236,
// N states, a VALU rewrite of v236 (another address).  The read must return
// the OLD address's data.  BUSY: 8 ds_read_b128 queued ahead of it, so the
// LDS unit is backed up when the victim read issues.
#define DS_WAR(NAME, BUSY, NOPS)                                                                  \
    __global__ __launch_bounds__(512) void NAME(float* out, int iters) {                          \
        __shared__ uint2 tab[1024];                                                                \
        for (int i = threadIdx.x; i < 1024; i += blockDim.x) tab[i] = make_uint2(7 * i + 1, 13 * i + 5); \
        __syncthreads();                                                                           \
        const int lane = threadIdx.x & 63;                                                         \
        const size_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;                       \
        const uint32_t base = (uint32_t)(uintptr_t)tab;                                            \
        const uint32_t a_old = base + 8 * ((lane * 5 + 3) & 511), a_new = base + 8 * (512 + lane);   \
        int nbad = 0;                                                                              \
        uint32_t first0 = 0, first1 = 0;                                                           \
        for (int it = 0; it < iters; ++it) {                                                       \
            uint32_t d0, d1;                                                                       \
            asm volatile("v_mov_b32 v236, %[ao]\n\ts_nop 7\n\t" BUSY                             \
                         "ds_read_b64 v[238:239], v236\n\t" NOPS                                 \
                         "v_mov_b32 v236, %[an]\n\t"                                              \
                         "s_waitcnt lgkmcnt(0)\n\ts_nop 3\n\t"                                   \
                         "v_mov_b32 %[d0], v238\n\tv_mov_b32 %[d1], v239"                        \
                         : [d0] "=&v"(d0), [d1] "=&v"(d1)                                          \
                         : [ao] "v"(a_old), [an] "v"(a_new), [b] "v"(base + 16 * lane)            \
                         : "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", \
                           "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", \
                           "v238", "v239", "memory");                                              \
            if (it == 0) {                                                                         \
                first0 = d0;                                                                       \
                first1 = d1;                                                                       \
            }                                                                                      \
            nbad += (d0 != first0) || (d1 != first1);                                              \
        }                                                                                          \
        out[(w * 64 + lane) * 2 + 0] = __uint_as_float(first0);                                    \
        out[(w * 64 + lane) * 2 + 1] = __uint_as_float(first1);                                    \
        out[(size_t)gridDim.x * (blockDim.x / 64) * 64 * 2 + w * 64 + lane] = (float)nbad;        \
    }
#define DS_BUSY                                                                                   \
    "ds_read_b128 v[220:223], %[b]\n\tds_read_b128 v[224:227], %[b] offset:1024\n\t"             \
    "ds_read_b128 v[228:231], %[b] offset:2048\n\tds_read_b128 v[232:235], %[b] offset:3072\n\t" \
    "ds_read_b128 v[220:223], %[b] offset:4096\n\tds_read_b128 v[224:227], %[b] offset:5120\n\t" \
    "ds_read_b128 v[228:231], %[b] offset:6144\n\tds_read_b128 v[232:235], %[b] offset:7168\n\t"
DS_WAR(ds_war_0, "", NOPS_0)
DS_WAR(ds_war_busy_0, DS_BUSY, NOPS_0)
DS_WAR(ds_war_busy_1, DS_BUSY, NOPS_1)
DS_WAR(ds_war_busy_4, DS_BUSY, NOPS_4)

// bf16 (the §13e2 DFT's instruction): checked against the nops-8 form and
// the old-operand product, both measured (no host reference)
PROBE_KERNEL(raw_bf_0, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_0 MFMA_BF DRAIN)
PROBE_KERNEL(raw_bf_1, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_1 MFMA_BF DRAIN)
PROBE_KERNEL(raw_bf_2, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_2 MFMA_BF DRAIN)
PROBE_KERNEL(raw_bf_8, SET_OLD "s_nop 7\n\t" PERM_NEW NOPS_8 MFMA_BF DRAIN)
PROBE_KERNEL(old_bf, SET_OLD "s_nop 7\n\t" MFMA_BF DRAIN)
PROBE_KERNEL(war_bf_0, SET_OLD "s_nop 7\n\t" MFMA_BF NOPS_0 MOV_NEW DRAIN)

// The compiler's own RAW schedule: B assembled by __builtin_amdgcn_perm, then
// the MFMA builtin (hipcc inserts the wait states it believes are needed)
__global__ __launch_bounds__(512) void raw_perm_compiler(const uint32_t* in, float* out, int iters) {
    const int lane = threadIdx.x & 63;
    const size_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    frag8 a, lo, hi;
    for (int q = 0; q < 4; ++q) {
        a[q] = in[lane * 4 + q];
        lo[q] = in[512 + lane * 4 + q];
        hi[q] = in[768 + lane * 4 + q];
    }
    int nbad = 0;
    float first[16];
    for (int it = 0; it < iters; ++it) {
        asm volatile("" : "+v"(lo), "+v"(hi));
        frag8 b;
        for (int q = 0; q < 4; ++q) b[q] = __builtin_amdgcn_perm(hi[q], lo[q], 0x05040100u);
        const f32x16 acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                                  __builtin_bit_cast(f16x8, b), f32x16{}, 0, 0, 0);
        if (it == 0)
            for (int r = 0; r < 16; ++r) first[r] = acc[r];
        for (int r = 0; r < 16; ++r) nbad += acc[r] != first[r];
    }
    for (int r = 0; r < 16; ++r) out[(w * 64 + lane) * 16 + r] = first[r];
    out[(size_t)gridDim.x * (blockDim.x / 64) * 64 * 16 + w * 64 + lane] = (float)nbad;
}

// host reference: D[i][j] = sum_k A[i][k] B[k][j] with the 32x32x16 layout:
// lane (j, half) holds A row j, k = 8 half + 0..7 (and B column j, same k);
// D register r of lane (j, half) is row (r & 3) + 8 (r >> 2) + 4 half, column j
static float h2f(uint16_t h) {
    const uint32_t s = (h >> 15) & 1, e = (h >> 10) & 31, m = h & 1023;
    float v;
    if (e == 0) v = ldexpf((float)m, -24);
    else v = ldexpf((float)(m | 1024), (int)e - 25);
    return s ? -v : v;
}

static void ref(const uint32_t* A, const uint32_t* Bf, float* D) {
    float a[32][16], b[16][32];
    for (int lane = 0; lane < 64; ++lane) {
        const int j = lane & 31, half = lane >> 5;
        for (int e = 0; e < 8; ++e) {
            const uint16_t av = (uint16_t)(A[lane * 4 + e / 2] >> (16 * (e & 1)));
            const uint16_t bv = (uint16_t)(Bf[lane * 4 + e / 2] >> (16 * (e & 1)));
            a[j][8 * half + e] = h2f(av);
            b[8 * half + e][j] = h2f(bv);
        }
    }
    for (int lane = 0; lane < 64; ++lane) {
        const int j = lane & 31, half = lane >> 5;
        for (int r = 0; r < 16; ++r) {
            const int i = (r & 3) + 8 * (r >> 2) + 4 * half;
            float s = 0.f;
            for (int k = 0; k < 16; ++k) s += a[i][k] * b[k][j];
            D[lane * 16 + r] = s;
        }
    }
}

typedef void (*kern_t)(const uint32_t*, float*, int);

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 1024, threads = 512, iters = argc > 2 ? atoi(argv[2]) : 64;
    const int waves = blocks * threads / 64;
    std::vector<uint32_t> in(1024);
    srand(7);
    auto small16 = [](int v) -> uint16_t {  // small integers: exact in fp16 and in fp32 sums
        const float f = (float)v;
        // fp16 bits of an integer |v| < 1024
        if (v == 0) return 0;
        const uint16_t s = v < 0 ? 0x8000 : 0;
        int m = abs(v), e = 0;
        while (m >= 2048) { m >>= 1; ++e; }
        int ex = 10;
        while ((1 << ex) > m) --ex;
        const uint16_t bits = (uint16_t)(((ex + 15) << 10) | ((m << (10 - ex)) & 1023));
        (void)f;
        return s | bits;
    };
    for (int i = 0; i < 1024; ++i) {
        const uint16_t x = small16((rand() % 15) - 7), y = small16((rand() % 15) - 7);
        in[i] = (uint32_t)x | ((uint32_t)y << 16);
    }
    // B "new" = perm(hi, lo, 0x05040100) = low halves of lo (bits 0-15) and hi (bits 16-31)
    std::vector<uint32_t> bnew(256), bold(in.begin() + 256, in.begin() + 512);
    for (int i = 0; i < 256; ++i) bnew[i] = (in[512 + i] & 0xFFFF) | (in[768 + i] << 16);
    std::vector<uint32_t> bmov(in.begin() + 512, in.begin() + 768);
    std::vector<float> d_old(1024), d_new(1024), d_mov(1024), d_hi(1024), d_dep(1024), d_depnew(1024);
    std::vector<float> d_hinew(1024), d_2hiold(1024), d_2hinew(1024);
    ref(in.data(), bold.data(), d_old.data());
    ref(in.data(), bnew.data(), d_new.data());
    ref(in.data(), bmov.data(), d_mov.data());
    std::vector<uint32_t> bhi(in.begin() + 768, in.begin() + 1024);
    ref(in.data(), bhi.data(), d_hi.data());
    for (int i = 0; i < 1024; ++i) {
        d_dep[i] = d_hi[i] + d_old[i];     // the dependent chain on the old B
        d_depnew[i] = d_hi[i] + d_mov[i];  // ... on the rewritten B (the hazard)
        d_hinew[i] = d_hi[i] + d_new[i];
        d_2hiold[i] = d_hi[i] + d_hi[i] + d_old[i];
        d_2hinew[i] = d_hi[i] + d_hi[i] + d_new[i];
    }
    uint32_t* din;
    float* dout;
    const size_t nout = (size_t)waves * 64 * 16 + (size_t)waves * 64;
    hipMalloc(&din, 4096);
    hipMalloc(&dout, nout * 4);
    hipMemcpy(din, in.data(), 4096, hipMemcpyHostToDevice);
    std::vector<float> out(nout);
    struct K {
        const char* name;
        kern_t k;
        int war;  // 0: want new (RAW), 1: want old (WAR), 2: dependent chain on the old B,
                  // 3: hi + old (perm rewrite), 4: 2 hi + old, 5: hi + new (RAW into the chain)
    } ks[] = {{"war_inter_perm_nops0", war_inter_perm_0, 3}, {"war_inter_perm_nops1", war_inter_perm_1, 3},
              {"war_inter_perm_nops4", war_inter_perm_4, 3}, {"war_inter_chain_nops0", war_inter_chain_0, 4},
              {"raw_inter_nops1", raw_inter_1, 5}, {"raw_inter_nops2", raw_inter_2, 5},
              {"war_busy_indep_nops0", war_busy_indep_0, 1}, {"war_busy_indep_nops2", war_busy_indep_2, 1},
              {"war_busy_dep_nops0", war_busy_dep_0, 2},     {"war_busy_dep_nops1", war_busy_dep_1, 2},
              {"war_busy_dep_nops2", war_busy_dep_2, 2},     {"war_busy_dep_nops4", war_busy_dep_4, 2},
              {"war_busy_dep_nops8", war_busy_dep_8, 2},     {"raw_busy_nops0", raw_busy_0, 0},
              {"raw_busy_nops1", raw_busy_1, 0},{"raw_perm_nops0", raw_perm_0, 0},   {"raw_perm_nops1", raw_perm_1, 0},
              {"raw_perm_nops2", raw_perm_2, 0},   {"raw_perm_nops3", raw_perm_3, 0},
              {"raw_perm_nops4", raw_perm_4, 0},   {"raw_perm_nops8", raw_perm_8, 0},
              {"raw_perm_compiler", raw_perm_compiler, 0},
              {"war_mov_nops0", war_mov_0, 1},     {"war_mov_nops1", war_mov_1, 1},
              {"war_mov_nops2", war_mov_2, 1},     {"war_mov_nops4", war_mov_4, 1},
              {"war_mov_nops8", war_mov_8, 1}};
    for (auto& k : ks) {
        hipMemset(dout, 0, nout * 4);
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("{\"probe\": \"%s\", \"error\": \"launch failed\"}\n", k.name);
            return 1;
        }
        hipMemcpy(out.data(), dout, nout * 4, hipMemcpyDeviceToHost);
        const float* want = k.war == 5 ? d_hinew.data() : k.war == 4 ? d_2hiold.data() : k.war == 3 ? d_dep.data()
                            : k.war == 2 ? d_dep.data() : k.war ? d_old.data() : d_new.data();
        const float* other = k.war == 5 ? d_dep.data() : k.war == 4 ? d_2hinew.data() : k.war == 3 ? d_hinew.data()
                             : k.war == 2 ? d_depnew.data() : k.war ? d_mov.data() : d_old.data();
        long ok = 0, wrong_other = 0, garbage = 0, unstable = 0;
        long bad_lane_hist[64] = {};
        for (int w = 0; w < waves; ++w)
            for (int lane = 0; lane < 64; ++lane) {
                bool all_ok = true, all_other = true;
                for (int r = 0; r < 16; ++r) {
                    const float v = out[((size_t)w * 64 + lane) * 16 + r];
                    all_ok &= v == want[lane * 16 + r];
                    all_other &= v == other[lane * 16 + r];
                }
                unstable += out[(size_t)waves * 64 * 16 + (size_t)w * 64 + lane] != 0.0f;
                if (all_ok) ++ok;
                else {
                    ++bad_lane_hist[lane];
                    if (all_other) ++wrong_other;
                    else ++garbage;
                }
            }
        printf("{\"probe\": \"%s\", \"lanes\": %ld, \"correct\": %ld, \"other_operand\": %ld, \"neither\": %ld, "
               "\"lanes_varying_over_iterations\": %ld, \"bad_lanes\": [",
               k.name, (long)waves * 64, ok, wrong_other, garbage, unstable);
        bool first = true;
        for (int l = 0; l < 64; ++l)
            if (bad_lane_hist[l]) {
                printf("%s%d", first ? "" : ",", l);
                first = false;
            }
        printf("]}\n");
        fflush(stdout);
    }
    // DS address WAR
    {
        typedef void (*dk_t)(float*, int);
        struct KD {
            const char* name;
            dk_t k;
        } kd[] = {{"ds_addr_war_nops0", ds_war_0}, {"ds_addr_war_busy_nops0", ds_war_busy_0},
                  {"ds_addr_war_busy_nops1", ds_war_busy_1}, {"ds_addr_war_busy_nops4", ds_war_busy_4}};
        const size_t nd = (size_t)waves * 64 * 3;
        std::vector<float> od(nd);
        for (auto& k : kd) {
            hipMemset(dout, 0, nd * 4);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, dout, iters);
            if (hipDeviceSynchronize() != hipSuccess) {
                printf("{\"probe\": \"%s\", \"error\": \"launch failed\"}\n", k.name);
                return 1;
            }
            hipMemcpy(od.data(), dout, nd * 4, hipMemcpyDeviceToHost);
            long ok = 0, newaddr = 0, other = 0, unstable = 0;
            long badl[64] = {};
            for (size_t i = 0; i < (size_t)waves * 64; ++i) {
                const int lane = (int)(i & 63);
                const int io = (lane * 5 + 3) & 511, in_ = 512 + lane;
                uint32_t d0, d1;
                memcpy(&d0, &od[i * 2], 4);
                memcpy(&d1, &od[i * 2 + 1], 4);
                if (d0 == (uint32_t)(7 * io + 1) && d1 == (uint32_t)(13 * io + 5)) ++ok;
                else {
                    ++badl[lane];
                    if (d0 == (uint32_t)(7 * in_ + 1) && d1 == (uint32_t)(13 * in_ + 5)) ++newaddr;
                    else ++other;
                }
                unstable += od[(size_t)waves * 64 * 2 + i] != 0.0f;
            }
            printf("{\"probe\": \"%s\", \"lanes\": %ld, \"correct\": %ld, \"new_address\": %ld, \"neither\": %ld, "
                   "\"lanes_varying_over_iterations\": %ld, \"bad_lanes\": [", k.name, (long)waves * 64, ok, newaddr,
                   other, unstable);
            bool fst = true;
            for (int l = 0; l < 64; ++l)
                if (badl[l]) {
                    printf("%s%d", fst ? "" : ",", l);
                    fst = false;
                }
            printf("]}\n");
            fflush(stdout);
        }
    }
    // bf16 forms against measured references
    auto run = [&](kern_t k, std::vector<float>& o) {
        hipMemset(dout, 0, nout * 4);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
        if (hipDeviceSynchronize() != hipSuccess) return false;
        o.resize(nout);
        hipMemcpy(o.data(), dout, nout * 4, hipMemcpyDeviceToHost);
        return true;
    };
    std::vector<float> r_new, r_old, o;
    if (!run(raw_bf_8, r_new) || !run(old_bf, r_old)) {
        printf("{\"probe\": \"bf16 refs\", \"error\": \"launch failed\"}\n");
        return 1;
    }
    struct KB {
        const char* name;
        kern_t k;
        int war;
    } kb[] = {{"raw_bf16_nops0", raw_bf_0, 0}, {"raw_bf16_nops1", raw_bf_1, 0}, {"raw_bf16_nops2", raw_bf_2, 0},
              {"war_bf16_nops0", war_bf_0, 1}};
    for (auto& k : kb) {
        if (!run(k.k, o)) {
            printf("{\"probe\": \"%s\", \"error\": \"launch failed\"}\n", k.name);
            return 1;
        }
        const std::vector<float>& want = k.war ? r_old : r_new;
        const std::vector<float>& other = k.war ? r_new : r_old;
        long ok = 0, wrong_other = 0, garbage = 0;
        for (size_t i = 0; i < (size_t)waves * 64; ++i) {
            bool a1 = true, a2 = true;
            for (int r = 0; r < 16; ++r) {
                a1 &= o[i * 16 + r] == want[i * 16 + r];
                a2 &= o[i * 16 + r] == other[i * 16 + r];
            }
            ok += a1;
            wrong_other += !a1 && a2;
            garbage += !a1 && !a2;
        }
        printf("{\"probe\": \"%s\", \"lanes\": %ld, \"correct\": %ld, \"other_operand\": %ld, \"neither\": %ld}\n",
               k.name, (long)waves * 64, ok, wrong_other, garbage);
        fflush(stdout);
    }
    return 0;
}
