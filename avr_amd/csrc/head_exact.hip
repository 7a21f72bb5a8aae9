// Fused signal head, output-rounding-exact form.
//
// The reference's signal network returns x = h W^T from a 16-bit network
// (tcnn's fp16, model.py:21-31, 176-180): the render sees every element of x
// ROUNDED to 16 bits (renderer_cpu.py:73,80,90 upcast it with .float()).  The
// linear-algebra head of head.hip sums exact products and never forms x, so
// it cannot reproduce that rounding.  This kernel forms x tile by tile on the
// matrix cores, rounds each element to the MLP's 16-bit type exactly as the
// unfused layer's output does (fp32 accumulation, one round to nearest even),
// and reduces it over rays on the spot:
//
//   z[b,s,t] = sum_{p < cnt[b,s,t]} ws[b,s,p] * round16( sum_k h[b,perm_p,s,k] W[t,k] )
//
// with the column's live rays sorted by delay (avr_head_sort: perm, ws and
// cnt[t] = number of rays with delay <= t), so the live part of the
// [rays x t] plane is a staircase.
//
// h stationary, W streamed (round 4).  A work item is (ray block, column):
// RAYS consecutive sorted rays of one column (b, s); each wave owns 32 of
// them and holds their h rows as the A operand of v_mfma_f32_32x32x16 for
// the whole item (K/16 fragments, 128 VGPRs at K = 512), loaded ONCE: whole
// 1 KiB rows by LDS-DMA through the (then idle) ring, then into registers
// (stationary.h).  The item sweeps t in tiles of 32 NC from its first ray's
// delay to the tail limit; W, shared by every column and resident in each
// XCD's L2, streams through an NB-tile LDS ring by LDS-DMA in B-fragment
// order (avr_head_pack_w_exact).  h crosses HBM once (268 MB at config 2);
// only W's tiles move through LDS-DMA.  A wave whose rays are not live yet in
// a 32-t group skips its chain (32 x 32 staircase granularity).
//
// Per tile every wave rounds, masks (p < cnt[t], select on the VALUE so an
// overflowed masked product cannot leak 0 * inf) and weights its 32 x 32
// products and sums them per lane in position order; the two lane halves are
// added, then the waves' partials in wave order.  Each item writes its own
// slab zpart[block][b][s][t] (zero outside its live range); avr_dft_phase_fwd
// sums the n_split slabs in a fixed order, so results are deterministic.
//
// Persistent workgroups (as many as fit: two per CU for 128-ray items) take
// items from eight work queues, one per XCD's share of the items, in
// block-major order (every column's first block first: the longest items
// first, the short ones fill the tail).  The next item's metadata (kept-ray
// count, rays, cnt, weights, first delay) is loaded while the current item
// computes, so an item's prologue is its rows' DMA and the first W tile.
#include "common.h"
#include "probe.h"
#include "stationary.h"

#include <algorithm>

using namespace avr;

AVR_PROBE_TU(avr_probe_set_exact)

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t frag8 __attribute__((ext_vector_type(4)));  // 8 packed 16-bit values

template <typename E>
__device__ __forceinline__ f32x16 mfma16(frag8 a, frag8 b, f32x16 c) {
    if constexpr (std::is_same<E, __half>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

// x rounded to the 16-bit type E (round to nearest even) and back: the value
// the unfused layer's 16-bit output holds
template <typename E>
__device__ __forceinline__ float round16(float x) {
    if constexpr (std::is_same<E, __half>::value)
        return __half2float(__float2half(x));
    else
        return __bfloat162float(__float2bfloat16(x));
}

// One 16-byte-per-lane LDS-DMA load: lane i's 16 bytes at g land at LDS byte
// address lds + 16 i.  Issued as inline asm so the compiler does not treat
// the in-flight DMA as an LDS write every later ds_read must wait for (with
// the builtin it inserts vmcnt(0) inside the MFMA chain); completion is
// waited for explicitly with counted vmcnt.
__device__ __forceinline__ void dma_row16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(g)
                 : "memory", "m0");
}

// s_waitcnt vmcnt(n) (expcnt / lgkmcnt not waited on; gfx9 encoding)
#define AVR_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14))

// s_waitcnt vmcnt(n) for a run-time n (one case per value; above 31 the
// wait is for 31, a longer wait than asked)
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
#define AVR_VMC(K) case K: AVR_VMCNT(K); break;
        AVR_VMC(0) AVR_VMC(1) AVR_VMC(2) AVR_VMC(3) AVR_VMC(4) AVR_VMC(5) AVR_VMC(6) AVR_VMC(7)
        AVR_VMC(8) AVR_VMC(9) AVR_VMC(10) AVR_VMC(11) AVR_VMC(12) AVR_VMC(13) AVR_VMC(14) AVR_VMC(15)
        AVR_VMC(16) AVR_VMC(17) AVR_VMC(18) AVR_VMC(19) AVR_VMC(20) AVR_VMC(21) AVR_VMC(22) AVR_VMC(23)
        AVR_VMC(24) AVR_VMC(25) AVR_VMC(26) AVR_VMC(27) AVR_VMC(28) AVR_VMC(29) AVR_VMC(30) AVR_VMC(31)
#undef AVR_VMC
        default: AVR_VMCNT(31); break;
    }
}

// largest T of the 8-wave and the 4-wave items (exact_shape)
constexpr int kExactMaxT[2] = {4096, 1024};

// threadIdx.x through an empty asm: in a persistent kernel's item loop, the
// per-lane values derived from it are formed where they are used instead of
// hoisted out of the loop and held in registers (or spilled) across it
__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// bytes of one 32-t W tile in fragment order: KSM k-steps x 64 lanes x 16 B
__host__ __device__ constexpr int xs_tile_bytes(int KSM) { return KSM * 1024; }
// wave partials: one buffer per tile in flight (tile i's in zr[i % 2] until
// the wave that sums it has read them, two barriers later)
constexpr int kPartBufs = 2;
// B fragments read ahead from the ring in an MFMA chain, and the MFMAs
// (each at least two instructions: the MFMA and a ring read) after which a
// fragment's register may be reused: 8 wait states
constexpr int kReadAhead = 8;
constexpr int kHold = 4;

__host__ __device__ constexpr size_t xs_lds_bytes(int KSM, int T, int waves, int rays, int nb, int nc) {
    return (size_t)nb * nc * xs_tile_bytes(KSM) + 4 * (size_t)((T + 3) / 4 * 4) + 4 * (size_t)rays +
           4 * (size_t)(kPartBufs * waves * 32 * nc) + 4 * (size_t)waves + 8;
}

// One work item: RAYS consecutive sorted rays of one column (b, s), WAVES
// waves of RPW = RAYS / WAVES rays (NQ = RPW / 32 MFMA A tiles each), a ring
// of NB W tiles.  <8, 256, 4>: one workgroup per CU (two waves per SIMD);
// <4, 128, 2>: half the item and ~70 KB of LDS, so two workgroups share a CU
// and one's prologue and barriers overlap the other's MFMA chains.
template <typename E, int KSM, int WAVES, int RAYS, int NB, int NC, bool ROWDMA>
__global__ __launch_bounds__(64 * WAVES, 2) void head_exact_kernel(
    avr_render_params pp, int B, int R, int K, const E* __restrict__ h, const frag8* __restrict__ Wf,
    const int* __restrict__ perm, const float* __restrict__ ws, const int* __restrict__ cnt,
    const int32_t* __restrict__ delay, float* __restrict__ zpart, int* __restrict__ queue, int nitems, int prio) {
    constexpr int NT = 64 * WAVES, TILE = NC * xs_tile_bytes(KSM);  // a tile: TT = 32 NC values of t
    constexpr int TT = 32 * NC;
    constexpr int RPW = RAYS / WAVES;    // rays per wave
    constexpr int NQ = RPW / 32;         // 32-ray A tiles per wave
    // W-tile DMA pieces (1 KiB each), issued by every wave inside the tile's
    // first live chain
    constexpr int DPW = NC * KSM / WAVES;  // pieces per wave and tile
    static_assert((NC * KSM) % WAVES == 0 && NQ == 1 && DPW * NB <= 63 && NT >= RAYS && KSM % DPW == 0, "shape");
    // the partial buffers zr[i % kPartBufs] written in iteration i are read
    // after its barrier; rewritten in iteration i + kPartBufs, past one more
    static_assert(kPartBufs == 2, "the tile loop's partial-buffer rotation assumes two buffers");
    AVR_PROBE_DECL;
    extern __shared__ __attribute__((aligned(16))) char lds_x[];
    const int T = pp.T, S = pp.n_samples;
    const int Tp = (T + 3) & ~3;
    char* ring = lds_x;                                         // [NB][TILE]
    int* cl = reinterpret_cast<int*>(lds_x + NB * TILE);        // cnt of the column [Tp]
    float* wl = reinterpret_cast<float*>(cl + Tp);              // weights of the item's rays [RAYS]
    float* zr = wl + RAYS;                                      // wave partials [kPartBufs][WAVES][TT]
    int* dstart = reinterpret_cast<int*>(zr + kPartBufs * WAVES * TT);  // first live t per wave [WAVES]
    int* qnext = dstart + WAVES;                                // claimed items [2]

    const int64_t ncol = (int64_t)B * S;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // static priority for the second-dispatched half of the waves (the
    // arbitration loser of every segment; MI355X_MICROARCH.md, two waves per SIMD)
    if (prio && wave >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
    const int ksn = K / 16;
    constexpr bool dma_rows = ROWDMA;  // K == 512: whole 1 KiB rows by LDS-DMA
    const uint32_t ring_lds = (uint32_t)(uintptr_t)ring;

    // ---- work queue: items x, x + 8, x + 16, ... (block-major: longest
    // first) are served by queue x = blockIdx.x % 8 to its G/8 workgroups;
    // claims 0, 1 and 2 of workgroup l are l, G/8 + l and 2 G/8 + l, later
    // ones come from the queue's counter (zeroed by the host before the
    // launch).  A claim is made two items ahead: thread 0 claims at the start
    // of item i, publishes it in LDS at the end of item i, and every thread
    // reads it at the end of item i + 1 (barriers in between; two slots).
    const int qx = blockIdx.x & 7, gq = gridDim.x >> 3, ql = blockIdx.x >> 3;
    int* qctr = queue + 32 * qx;  // one 128-byte line per counter
    auto item_of = [&](int claim) { return qx + 8 * claim; };

    // metadata of an item, loaded one item ahead: every load independent of
    // the others (a claim past the last item loads a clamped, valid address),
    // all of them vector loads (lane-varying addresses): a scalar load in
    // flight would hold up every lgkmcnt wait of the LDS traffic meanwhile
    constexpr int CLN = (kExactMaxT[WAVES == 4] + NT - 1) / NT;  // cnt values per thread
    struct Meta {
        int item, nk, ray, dly;
        int clv[CLN];
        float wsv;
    };
    auto load_meta = [&](int item, Meta& m) {
        const int tid = opaque_tid();
        m.item = item;
        const int it = min(item, nitems - 1);
        const int64_t col = (int64_t)it % ncol;
        const int blk = (int)((int64_t)it / ncol);
        const int* cc = cnt + col * T;
        m.nk = cc[T - 1 - (tid >> 12)];  // kept rays of the column (tid < 4096: T - 1)
        // the ray of each lane's sorted position (avr_head_sort leaves ray 0
        // past the kept rays: a valid row, masked by weight and count)
        m.ray = perm[col * R + min(blk * RAYS + RPW * wave + (tid & 31), R - 1)];
#pragma unroll
        for (int u = 0; u < CLN; ++u) m.clv[u] = cc[min(tid + NT * u, T - 1)];
        m.wsv = ws[col * R + min(blk * RAYS + tid, R - 1)];
    };
    // each wave's first live t: the delay of its first sorted ray (sorted by
    // delay, so cnt[t] > pw from that t on; lane 0's value); issued once
    // m.ray has landed
    auto load_dly = [&](Meta& m) {
        const int it = min(m.item, nitems - 1);
        const int64_t col = (int64_t)it % ncol;
        const int s = (int)(col % S), b = (int)(col / S);
        m.dly = delay[((int64_t)b * R + m.ray) * S + s];
    };
    // wait for a prefetched item's loads here (empty asm uses): the compiler
    // places its wait at the first use, which must not be at the next item's
    // start, behind that item's own fresh loads
    auto touch = [&](Meta& m) {
        asm volatile("" ::"v"(m.nk), "v"(m.ray), "v"(m.dly), "v"(m.wsv));
#pragma unroll
        for (int u = 0; u < CLN; ++u) asm volatile("" ::"v"(m.clv[u]));
    };

    Meta cur, nx;
    int claim = 0;
    int item = item_of(ql), nxt = item_of(gq + ql);
    load_meta(item, cur);
    load_dly(cur);
    if (threadIdx.x == 0) qnext[1] = item_of(2 * gq + ql);
    __syncthreads();
    for (int iter = 0; item < nitems; ++iter) {
        AVR_PROBE_DECL;
        const int tid = opaque_tid();
        const int lane = tid & 63, half = lane >> 5, j = lane & 31;
        const int col = item % (int)ncol;  // items < 2^31 (checked by the host)
        const int blk = item / (int)ncol;
        const int s = col % S, b = col / S;
        const int lim = tail_limit(pp, s);
        float* zc = zpart + ((int64_t)blk * ncol + col) * T;
        const int p0 = blk * RAYS;
        const int pw = p0 + RPW * wave;
        const int nk = __builtin_amdgcn_readfirstlane(cur.nk);
        // a claim two items ahead (thread 0's register; defined only by the
        // atomic, so no re-initialisation at the loop top waits for the last
        // one: a write-after-write behind a returning atomic costs a full
        // vmcnt(0) there)
        if (tid == 0) {
            // the counter's offset through an empty asm: not provably uniform,
            // so the compiler's wave-aggregating atomic rewrite (which waits for
            // the result on the spot) does not apply; the wait is at the use
            int zero = 0;
            asm volatile("" : "+v"(zero));
            claim = __hip_atomic_fetch_add(qctr + zero, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool dly_issued = false, touched = false, published = false;
        if (p0 >= nk || lim <= 0) {
            load_meta(nxt, nx);
            for (int t = tid; t < T; t += NT) zc[t] = 0.0f;
            load_dly(nx);
            dly_issued = true;
        } else {
            // ---- prologue: the wave's rows by LDS-DMA through the (idle) ring
            const E* hrow = h + (((int64_t)b * R + cur.ray) * S + s) * K;
            frag8 a[NQ][KSM];
            if (AVR_PROBE_SKIP(4)) {
#pragma unroll
                for (int ks = 0; ks < KSM; ++ks) a[0][ks] = frag8{(uint32_t)ks, 0u, 0u, 0u};
#pragma unroll
                for (int ks = 0; ks < KSM; ++ks) asm volatile("" : "+v"(a[0][ks]));
            } else if constexpr (dma_rows) {
                // every fragment defined before the lane-masked round writes:
                // an undefined start would let the compiler carry the previous
                // item's fragments into this item's prologue (128 more VGPRs)
#pragma unroll
                for (int ks = 0; ks < KSM; ++ks) a[0][ks] = frag8{0u, 0u, 0u, 0u};
                stat_issue_round(reinterpret_cast<const uint16_t*>(hrow), ring + wave * 16384, 0);
                stat_issue_round(reinterpret_cast<const uint16_t*>(hrow), ring + wave * 16384, 1);
                AVR_PROBE_MARK(8);
                stat_finish_rows512(reinterpret_cast<frag8_t(&)[32]>(a[0]), reinterpret_cast<const uint16_t*>(hrow),
                                    ring + wave * 16384);
            } else {
#pragma unroll
                for (int ks = 0; ks < KSM; ++ks)
                    a[0][ks] = *reinterpret_cast<const frag8*>(hrow + 8 * half + 16 * min(ks, ksn - 1));
#pragma unroll
                for (int ks = 0; ks < KSM; ++ks)
                    if (ks >= ksn) a[0][ks] = frag8{0u, 0u, 0u, 0u};
#pragma unroll
                for (int ks = 0; ks < KSM; ++ks) asm volatile("" ::"v"(a[0][ks]));
                AVR_VMCNT(0);
            }
            AVR_PROBE_MARK(9);
            // cnt, the item's weights and the waves' first live t into LDS
#pragma unroll
            for (int u = 0; u < CLN; ++u) {
                const int t = tid + NT * u;
                if (t < T) cl[t] = cur.clv[u];
            }
            if (tid < RAYS) wl[tid] = p0 + tid < nk ? cur.wsv : 0.0f;
            if (lane == 0) dstart[wave] = pw < nk ? cur.dly : 1 << 30;
            // staging area free (the ring may fill); cl, wl, dstart written.  A
            // bare barrier: nothing in flight on the vector-memory counter is
            // waited for (the claim's atomic)
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
            AVR_PROBE_MARK(10);
            const int tb = dstart[0] / TT;       // first tile with a live ray of the item
            const int te = (lim + TT - 1) / TT;  // tiles holding t < lim
            // W tile tau into ring slot `slot`: this wave's pieces
            auto issue = [&](int tau, int slot) {
                if (AVR_PROBE_SKIP(1)) return;
                const char* src =
                    reinterpret_cast<const char*>(Wf) + (int64_t)tau * TILE + wave * DPW * 1024 + 16 * lane;
                const uint32_t dst = ring_lds + slot * TILE + wave * DPW * 1024;
                for (int d = 0; d < DPW; ++d) dma_row16(src + d * 1024, dst + d * 1024);
            };
            for (int i = 0; i < NB - 1; ++i)
                if (tb + i < te) issue(tb + i, i);
            // the next item's metadata: in flight under this item, younger than
            // the first tiles, so only the tiles are waited for here
            load_meta(nxt, nx);
            AVR_VMCNT(CLN + 3);  // the first tiles and the (older) claim have landed
            if (tid == 0) {
                // published now, not at the item's end: no returning atomic is
                // in flight at the loop's back edge (the compiler would wait for
                // every store of the item there).  Slot iter & 1 was last read
                // before this item's first barrier
                qnext[iter & 1] = item_of(3 * gq + claim);
                published = true;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
            AVR_PROBE_MARK(2);
#ifdef AVR_PHASE_PROBES
            probe_w[12] = te - tb;                                   // tiles of the item
            probe_w[13] = (uint64_t)(dstart[wave] < (1 << 30) ? (lim - dstart[wave] + 31) / 32 : 0);  // wave's live tiles
            probe_w[14] = blockIdx.x;
#endif

            // the wave's 32 rays against 32-t column group c of the tile in
            // ring slot `slot`: one MFMA chain over K (A from registers, B read
            // from the ring D k-steps ahead), then the epilogue (rounded,
            // masked by value: p < cnt[t], weighted, summed per lane in row order)
            const float* wq = wl + RPW * wave + 4 * half;
            // The next W tile's DMA pieces (dtile >= 0) are issued inside the
            // chain, one every KSM / DPW MFMAs: issued back to back before it,
            // each stalls the wave ~100 cycles behind the previous one
            // (tools/probe_phases.py), while between MFMAs the stall overlaps
            // the matrix pipe.
            // the wave's DMA pieces of tile dtile (if >= 0) issued inside the
            // chain, one every KSM / DPW MFMAs
            auto chain = [&](int slot, int c, int dtile, int dslot) {
                const char* bsrc = ring + slot * TILE + c * xs_tile_bytes(KSM) + 16 * lane;
                constexpr int D = KSM < kReadAhead ? KSM : kReadAhead;  // B fragments read ahead
                // a ring of D + kHold fragments: the read for k-step ks + D
                // (issued after MFMA ks) goes into the slot of k-step
                // ks - kHold, and the fragments of k-steps ks - kHold + 1 ..
                // ks are used once more after MFMA ks (program order fixed by
                // the sched_barrier), so the read is never allocated onto the
                // B register of one of the last kHold MFMAs, which may still
                // wait in the matrix pipe's queue (common.h, §15a)
                constexpr int RS = D + kHold;
                constexpr int DSTEP = KSM / DPW;      // MFMAs per DMA piece
                frag8 bw[RS];
#pragma unroll
                for (int u = 0; u < D; ++u) bw[u] = *reinterpret_cast<const frag8*>(bsrc + u * 1024);
                f32x16 acc = f32x16{};
                const char* dsrc =
                    reinterpret_cast<const char*>(Wf) + (int64_t)dtile * TILE + wave * DPW * 1024 + 16 * lane;
                const uint32_t ddst = ring_lds + dslot * TILE + wave * DPW * 1024;
                const bool dma = dtile >= 0 && !AVR_PROBE_SKIP(1);
#pragma unroll
                for (int ks = 0; ks < KSM; ++ks) {
                    acc = mfma16<E>(a[0][ks], bw[ks % RS], acc);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < kHold; ++q)
                        if (ks >= q) keep_live(bw[(ks - q) % RS]);
                    if (ks + D < KSM) bw[(ks + D) % RS] = *reinterpret_cast<const frag8*>(bsrc + (ks + D) * 1024);
                    if (ks % DSTEP == 0 && dma) dma_row16(dsrc + (ks / DSTEP) * 1024, ddst + (ks / DSTEP) * 1024);
                }
                mfma_queue_wait();
#pragma unroll
                for (int u = 0; u < RS; ++u) keep_live(bw[u]);
                return acc;
            };
            auto epi = [&](const f32x16& acc, int tau, int c) {
                if (AVR_PROBE_SKIP(2)) return acc[0] + acc[15];
                // register r of acc is row (r & 3) + 8 (r >> 2) + 4 half of the
                // wave's rays, column t = TT tau + 32 c + j
                const int t0 = TT * tau + 32 * c;
                const int t = t0 + j;
                const int full = __builtin_amdgcn_readfirstlane((t0 + 31 < lim) ? cl[t0] : 0);
                float z = 0.0f;
                if (pw + 32 <= full) {  // every (ray, t) pair of the group is live
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const float4 w4 = *reinterpret_cast<const float4*>(wq + 8 * g);
                        z = fmaf(w4.x, round16<E>(acc[4 * g + 0]), z);
                        z = fmaf(w4.y, round16<E>(acc[4 * g + 1]), z);
                        z = fmaf(w4.z, round16<E>(acc[4 * g + 2]), z);
                        z = fmaf(w4.w, round16<E>(acc[4 * g + 3]), z);
                    }
                } else {
                    const int ct = t < lim ? cl[min(t, T - 1)] : 0;
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const float4 w4 = *reinterpret_cast<const float4*>(wq + 8 * g);
                        const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float v = round16<E>(acc[4 * g + e]);
                            z = fmaf(wv[e], (pw + 8 * g + 4 * half + e < ct) ? v : 0.0f, z);
                        }
                    }
                }
                return z;
            };
            // a chain's per-lane sum, lower + upper lane half (rows 4 half +
            // ...; the same association in every lane), into the partials of
            // buffer `buf`
            auto put = [&](float zlc, int buf, int c) {
                const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(zlc), __float_as_uint(zlc), false,
                                                                false);
                const float v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
                if (half == 0) zr[buf * (WAVES * TT) + wave * TT + 32 * c + j] = v;
            };
            // the wave partials of tile tau (buffer `buf`), in wave order
            auto sum_tile = [&](int tau, int buf) {
                if (lane < TT) {
                    const float* zz = zr + buf * (WAVES * TT) + lane;
                    float v = zz[0];
#pragma unroll
                    for (int w = 1; w < WAVES; ++w) v += zz[TT * w];
                    const int t = TT * tau + lane;
                    if (t < T) zc[t] = v;
                }
            };
            // the wave that sums (and stores) tile i's partials right after
            // the barrier of iteration i
            auto summer = [&](int m) { return m % WAVES; };
            for (int tau = tb; tau < te; ++tau) {
                const int i = tau - tb;
                AVR_PROBE_BEGIN(comp);
                // tile tau + NB - 1 into the slot tile tau - 1 left: inside the
                // first live group's chain, else here
                const int dtile = tau + NB - 1 < te ? tau + NB - 1 : -1;
                const int dslot = (i + NB - 1) % NB;
                bool issued = false;  // dtile's pieces issued
                float zl[NC];
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    // group c holds a live ray of the wave from the wave's first
                    // live t on (cnt is nondecreasing in t), nothing at or past lim
                    const int t0 = TT * tau + 32 * c;
                    zl[c] = 0.0f;
                    if (t0 + 31 >= dstart[wave] && t0 < lim) {
                        const f32x16 acc = chain(i % NB, c, issued ? -1 : dtile, dslot);
                        issued = true;
                        zl[c] = epi(acc, tau, c);
                    }
                }
                if (dtile >= 0 && !issued) issue(dtile, dslot);
                AVR_PROBE_END(comp, 6);
#pragma unroll
                for (int c = 0; c < NC; ++c) put(zl[c], i % kPartBufs, c);
                AVR_PROBE_BEGIN(dma);
                if (tau + 1 < te) {
                    // this wave's pieces of tile tau+1 have landed.  Younger in
                    // vmcnt: the ring's later tiles and this wave's partial
                    // stores since tile tau+1 was issued (a wave stores after
                    // the barrier of iteration m when wave == summer(m)), so no
                    // store in flight is waited for
                    int st = 0;
                    for (int m = max(0, i + 2 - NB); m < i; ++m) st += (wave == summer(m));
                    wait_vm(min(NB - 2, te - 2 - tau) * DPW + st);
                }
                if (i == min(1, te - 1 - tb)) {
                    // the next item's delay (its ray has landed by now): older
                    // than the tiles issued from the next iteration on
                    load_dly(nx);
                    dly_issued = true;
                }
                if (tau == te - 1) {  // before the last partial store: nothing young to wait for
                    touch(nx);
                    touched = true;
                }
                AVR_PROBE_END(dma, 4);
                AVR_PROBE_BEGIN(bar);
                __builtin_amdgcn_s_waitcnt(0xC07F);  // every LDS access of tile tau (and the partials) done
                __builtin_amdgcn_s_barrier();
                AVR_PROBE_END(bar, 5);
                if (wave == summer(i)) sum_tile(tau, i % kPartBufs);
            }
            // zero outside the item's tiles (after the tiles: no wait above
            // includes these stores)
            for (int t = tid; t < T; t += NT)
                if (t < TT * tb || t >= TT * te) zc[t] = 0.0f;
            // the next item's prologue rewrites the ring and the LDS metadata:
            // every wave has passed the last tile's barrier, after which only
            // the partials zr are read (rewritten after two more barriers)
        }
        if (!dly_issued) load_dly(nx);
        if (!touched) touch(nx);
        if (tid == 0 && !published) qnext[iter & 1] = item_of(3 * gq + claim);
        if (p0 >= nk || lim <= 0) __syncthreads();  // every item has a barrier between the qnext accesses
        AVR_PROBE_FLUSH((int64_t)item * WAVES + wave);
        item = nxt;
        nxt = qnext[(iter + 1) & 1];
        cur = nx;
    }
}

// W [T][K] -> Wf: for t-tile tau and k-step ks, the 64 lanes' 16-byte B
// fragments of v_mfma_f32_32x32x16 (lane (j, half): W[32 tau + j][16 ks + 8 half
// + 0..7]) contiguous, zero past T and K
template <typename E>
__global__ __launch_bounds__(256) void head_pack_exact_kernel(int T, int K, int KSM, const uint16_t* __restrict__ W,
                                                              frag8* __restrict__ Wf, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int lane = (int)(i & 63);
        const int64_t r = i >> 6;
        const int ks = (int)(r % KSM);
        const int tau = (int)(r / KSM);
        const int t = 32 * tau + (lane & 31), k0 = 16 * ks + 8 * (lane >> 5);
        frag8 v = frag8{0u, 0u, 0u, 0u};
        if (t < T && k0 < K) v = *reinterpret_cast<const frag8*>(W + (int64_t)t * K + k0);
        Wf[i] = v;
    }
}

constexpr int kExactQueueInts = 256;  // 8 work-queue counters, one 128-byte line each

int exact_ksm(int K) { return K <= 128 ? 8 : (K <= 256 ? 16 : 32); }

// Work-item shape.  K = 512 (the reference networks' width, rows by
// LDS-DMA): 256 rays, one workgroup of eight waves per CU, 64-t tiles (two
// MFMA chains per wave between barriers), 239 vs 248 us for the 128-ray form
// per config-2 fp16 render (tools/ab_shapes.py, round 4).  Otherwise 128
// rays and two workgroups per CU where the DFT's slab count allows (<= 2048
// rays) and two ~70 KB LDS images fit (T <= 1024); 256 rays with 32-t tiles
// beyond.  AVR_EXACT_RAYS_PROBE / AVR_EXACT_TT_PROBE override it in the probe
// builds (csrc/probe.h).
struct ExactShape {
    int rays;
    bool tt64;
};

ExactShape exact_shape(int R, int T, int K) {
    ExactShape sh{(R <= 16 * 128 && T <= 1024) ? 128 : 256, false};
    if (K == 512) sh = {256, true};
    if (const char* e = AVR_PROBE_ENV("AVR_EXACT_RAYS_PROBE")) sh.rays = atoi(e) == 256 ? 256 : 128;
    if (const char* e = AVR_PROBE_ENV("AVR_EXACT_TT_PROBE")) sh.tt64 = atoi(e) == 64;
    if (sh.rays == 128 || K != 512) sh.tt64 = false;
    return sh;
}

int exact_check(const avr_render_params* p, int32_t K, int32_t dtype) {
    AVR_REQUIRE(p, "avr_head_fwd_exact: bad args");
    AVR_REQUIRE(dtype == AVR_DTYPE_F16 || dtype == AVR_DTYPE_BF16, "avr_head_fwd_exact: h/W must be fp16 or bf16");
    if (K % 16 != 0 || K < 16 || K > 512) return fail(AVR_E_CONFIG, "exact head: K must be a multiple of 16, <= 512");
    const int R = n_rays(*p);
    AVR_REQUIRE(R >= 1 && R <= 16 * 256 && p->T >= 2 && p->T <= 4096 && p->n_samples >= 1,
                "avr_head_fwd_exact: shape out of range (<= 4096 rays per shard, T <= 4096)");
    return 0;
}

// LDS of the launch avr_head_fwd_exact makes for (R, T, K): the W ring, the
// column's cnt, the item's weights and the wave partials (<= 160 KiB)
size_t exact_lds(int R, int T, int K) {
    const int KSM = exact_ksm(K);
    const ExactShape sh = exact_shape(R, T, K);
    if (sh.rays == 128) return xs_lds_bytes(KSM, T, 4, 128, 2, 1);
    if (sh.tt64) return xs_lds_bytes(KSM, T, 8, 256, 2, 2);
    return xs_lds_bytes(KSM, T, 8, 256, 4, 1);
}

int exact_splits(int R, int T, int K) {
    const int rays = exact_shape(R, T, K).rays;
    const int nb = (R + rays - 1) / rays;
    int n = 1;
    while (n < nb) n *= 2;
    return n;
}

template <typename Kern>
void allow_lds(Kern k, size_t lds) {
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

}  // namespace

extern "C" int avr_head_exact_layout(const avr_render_params* p, int32_t B, int32_t K, int32_t dtype,
                                     int32_t* n_split, int64_t* wpack_bytes) {
    AVR_REQUIRE(B >= 1 && n_split && wpack_bytes, "avr_head_exact_layout: bad args");
    if (int e = exact_check(p, K, dtype)) return e;
    if (exact_lds(n_rays(*p), p->T, K) > 160 * 1024)
        return fail(AVR_E_CONFIG, "exact head: LDS image above 160 KiB for this shape");
    *n_split = exact_splits(n_rays(*p), p->T, K);
    // whole 64-t tile pairs (a 64-t tile reads two consecutive 32-t tiles), zero past T
    *wpack_bytes = (int64_t)((p->T + 63) / 64) * 2 * xs_tile_bytes(exact_ksm(K));
    return 0;
}

extern "C" int avr_head_pack_w_exact(const avr_render_params* p, int32_t K, const void* W, int32_t dtype,
                                     void* Wf, void* stream) {
    AVR_REQUIRE(W && Wf, "avr_head_pack_w_exact: bad args");
    if (int e = exact_check(p, K, dtype)) return e;
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(W) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0,
                "avr_head_pack_w_exact: W and Wf must be 16-byte aligned");
    const int T = p->T, KSM = exact_ksm(K);
    const int64_t n = (int64_t)((T + 63) / 64) * 2 * KSM * 64;
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(head_pack_exact_kernel<__half>, dim3(blocks), dim3(256), 0, as_stream(stream), T, (int)K,
                       KSM, (const uint16_t*)W, (frag8*)Wf, n);
    return check_launch("avr_head_pack_w_exact");
}

extern "C" int avr_head_fwd_exact(const avr_render_params* p, int32_t B, int32_t K, const void* h, const void* Wf,
                                  int32_t dtype, const int32_t* perm, const float* ws, const int32_t* cnt,
                                  const int32_t* delay, int32_t n_split, float* zpart, int32_t* queue,
                                  void* stream) {
    AVR_REQUIRE(p && B >= 1 && h && Wf && perm && ws && cnt && delay && zpart && queue,
                "avr_head_fwd_exact: bad args");
    if (int e = exact_check(p, K, dtype)) return e;
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(h) % 16 == 0 && reinterpret_cast<uintptr_t>(Wf) % 16 == 0,
                "avr_head_fwd_exact: h and Wf must be 16-byte aligned");
    const int R = n_rays(*p), S = p->n_samples, T = p->T;
    AVR_REQUIRE(n_split == exact_splits(R, T, K), "avr_head_fwd_exact: n_split must be avr_head_exact_layout's");
    if (exact_lds(R, T, K) > 160 * 1024)
        return fail(AVR_E_CONFIG, "exact head: LDS image above 160 KiB for this shape");
    const int64_t items = (int64_t)n_split * B * S;
    AVR_REQUIRE(items < (1ll << 31), "avr_head_fwd_exact: too many columns");
    const int KSM = exact_ksm(K);
    hipStream_t st = as_stream(stream);
    const ExactShape shape = exact_shape(R, T, K);
    const bool small = shape.rays == 128, tt64 = shape.tt64;
    // s_setprio 1 for waves 4-7 of the 8-wave items: 234.0 vs 239.8 us per
    // config-2 fp16 fused render (tools/ab_shapes.py, 5 interleaved rounds);
    // the 4-wave items (two workgroups per CU) lose with it (252 vs 244)
    int prio = small ? 0 : 1;
    if (const char* pe = AVR_PROBE_ENV("AVR_EXACT_PRIO_PROBE")) prio = atoi(pe);
    auto run = [&](auto e_tag) {
        using E = decltype(e_tag);
        auto go = [&](auto kern, int ksm, int waves, int rays, int nb, int nc, const void* hv) {
            const size_t lds = xs_lds_bytes(ksm, T, waves, rays, nb, nc);
            allow_lds(kern, lds);
            // persistent workgroups: as many as fit on the chip at once (a
            // multiple of 8: one work queue per XCD), at most one per 8 items
            int per_cu = 1;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * waves, lds) != hipSuccess ||
                per_cu < 1)
                per_cu = 1;
            const int64_t gq = std::min<int64_t>((int64_t)device_cus() * per_cu / 8, (items + 7) / 8);
            const int grid = 8 * (int)std::max<int64_t>(gq, 1);
            (void)hipMemsetAsync(queue, 0, kExactQueueInts * sizeof(int32_t), st);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), lds, st, *p, (int)B, R, (int)K, (const E*)hv,
                               (const frag8*)Wf, perm, ws, cnt, delay, zpart, (int*)queue, (int)items, prio);
        };
        const bool rowdma = K == 512;
        if (small) {
            if (KSM == 8) go(head_exact_kernel<E, 8, 4, 128, 2, 1, false>, 8, 4, 128, 2, 1, h);
            else if (KSM == 16) go(head_exact_kernel<E, 16, 4, 128, 2, 1, false>, 16, 4, 128, 2, 1, h);
            else if (rowdma) go(head_exact_kernel<E, 32, 4, 128, 2, 1, true>, 32, 4, 128, 2, 1, h);
            else go(head_exact_kernel<E, 32, 4, 128, 2, 1, false>, 32, 4, 128, 2, 1, h);
        } else if (tt64 && rowdma) {
            go(head_exact_kernel<E, 32, 8, 256, 2, 2, true>, 32, 8, 256, 2, 2, h);
        } else {
            if (KSM == 8) go(head_exact_kernel<E, 8, 8, 256, 4, 1, false>, 8, 8, 256, 4, 1, h);
            else if (KSM == 16) go(head_exact_kernel<E, 16, 8, 256, 4, 1, false>, 16, 8, 256, 4, 1, h);
            else if (rowdma) go(head_exact_kernel<E, 32, 8, 256, 4, 1, true>, 32, 8, 256, 4, 1, h);
            else go(head_exact_kernel<E, 32, 8, 256, 4, 1, false>, 32, 8, 256, 4, 1, h);
        }
    };
    if (dtype == AVR_DTYPE_F16)
        run(__half{});
    else
        run(__hip_bfloat16{});
    return check_launch("avr_head_fwd_exact");
}
