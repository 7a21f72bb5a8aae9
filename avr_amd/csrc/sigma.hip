// Fused sigma networks (a5/a6): the width-128 bias-free ReLU MLPs the
// reference runs as tcnn FullyFusedMLP (sigma encoder + decoder,
// model.py:117-121, 146-150 / 267-277; configs avr_meshrir.yml:70-84,
// avr_raf_*.yml:89-101), plus the concatenation of the signal network's input
// (model.py:221 / 325), in ONE kernel for inference.
//
// Per sample n (262144 per config-2 pose):
//   AVRModel (variant 0):
//     h = relu(W3 relu(W2 relu(W1 relu(W0 e))))   e = pos_enc[n] (40)
//     sigma_feat = W3' ...                         (encoder output, 128, linear)
//     a = W7 relu(W6 relu(W5 relu(W4 relu(sigma_feat))))    (decoder, -> 1)
//     attn = |leaky_relu(a)|,  base[n] = [sigma_feat | dir_enc[ray] | tx_enc[pose]]
//   AVRModel_complex (variant 1):
//     rf = relu(W3 relu(W2 relu(W1 relu(W0 [pos_e[n] | txp_e[pose]]))))   (-> 256)
//     a = W5 relu(W4 rf),  attn = |leaky_relu(a, slope)|,
//     base[n] = [rf | dir[ray] | txdir[pose] | pos_sig[n] | txpos_sig[pose]]
//
// Unfused, this is 8 GEMMs whose [N,128] bf16 activations each make an HBM
// round trip, plus the concatenation copies (~0.35 ms per config-2 pose).
// Here activations never leave registers: every layer is computed TRANSPOSED,
// Y^T = W X^T, with v_mfma_f32_32x32x16_bf16 (A = weight fragment, B =
// activation fragment; sample on the lane).  The 32x32 fp32 result has its
// sample column on the lane and its output rows in the 16 registers, which is
// exactly the B-operand layout of the next layer's k-steps (registers 8s..8s+7
// = k-step s, cdna_hip_programming.md §3 "accumulator tile as the next MFMA's
// operand"); the k permutation that implies is folded into the packed weight
// fragments on the host (avr_amd/sigma.py), so the chain needs no LDS and no
// lane movement.  Weights (216-256 KB per net, bf16) stream through two 32 KB
// LDS buffers, one chunk (a layer or half a layer) each, one barrier per
// chunk, the next chunk's global loads in flight under the current chunk's
// MFMAs; every wave reads one 16-byte fragment per NT MFMAs with
// conflict-free ds_read_b128.
//
// Rounding is the unfused 16-bit path's: fp32 accumulation, activations in
// the MLP dtype E (bf16, or fp16 = tcnn's precision, model.py:21-31; ReLU
// before or after the rounding is the same), the decoder output rounded to E
// before leaky_relu (computed in fp32, rounded to E) and abs.  Fragments are
// carried as raw dwords; E only decides the conversions and the MFMA
// (v_mfma_f32_32x32x16_bf16 / _f16).
#include "common.h"
#include "probe.h"

using namespace avr;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef u32x4v frag8;  // 8 packed 16-bit values (one MFMA operand per lane)

// the 16-bit MLP element types: bf16 (__bf16) or fp16 (_Float16)
template <typename E>
__device__ __forceinline__ f32x16 mfma16(frag8 a, frag8 b, f32x16 c) {
    if constexpr (std::is_same<E, _Float16>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

constexpr int kChunk = 32768;  // bytes of packed fragments per LDS stage
constexpr int kFrag = 1024;    // one fragment: 64 lanes x 8 bf16

struct Src {
    const void* p;
    int dtype;
    int rows_div;
    int64_t lm_rows;  // 0: row-major [rows][width]; else level-major [width/2][lm_rows][2]
};

struct Args {
    int64_t N;
    Src in0, in1;
    int n_extra;
    Src extra[AVR_SIGMA_MAX_EXTRA];
    int extra_col[AVR_SIGMA_MAX_EXTRA];
    int extra_width[AVR_SIGMA_MAX_EXTRA];
    const char* wpack;
    uint16_t* base;  // E bits
    int ldb;
    uint16_t* attn;  // E bits
    float slope;
    const float* bias;  // variant 2: per-group bias of the signal network's first layer [rows][512]
    int bias_div;
    int nt_store;       // variant 2: streaming (non-temporal) h1 stores
};

// two fp32 -> a dword of two E (round to nearest even)
template <typename E>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    if constexpr (std::is_same<E, _Float16>::value)
        return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, f16x2));
    else
        return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, bf16x2));
}
// fp32 -> E -> fp32 (the 16-bit rounding of one value) and its bits
template <typename E>
__device__ __forceinline__ float round16(float v) { return (float)(E)v; }
template <typename E>
__device__ __forceinline__ uint16_t bits16(float v) { return __builtin_bit_cast(uint16_t, (E)v); }

// ReLU of two packed 16-bit floats (v_pk_max_i16 with 0: a set sign bit is a
// negative int16; bf16 and fp16 alike).  One VALU op per two values; a NaN
// with the sign bit set becomes 0.
// (IEEE-754 2019 maximum: NaN passes, one v_maximum3_f32 instead of a
// compare and a select)
#if AVR_SIGMA_RELU_SELECT  // (the round-4 form, for A/B: v_cmp + v_cndmask)
__device__ __forceinline__ float relu(float v) { return v < 0.0f ? 0.0f : v; }
#else
__device__ __forceinline__ float relu(float v) { return __builtin_elementwise_maximum(v, 0.0f); }
#endif

__device__ __forceinline__ uint32_t relu16x2(uint32_t u) {
    const s16x2 r = __builtin_elementwise_max(__builtin_bit_cast(s16x2, u), (s16x2){0, 0});
    return __builtin_bit_cast(uint32_t, r);
}

// 8 consecutive features (fp16 or fp32) of row `row` starting at `col` -> E
template <typename E>
__device__ __forceinline__ frag8 load8(const Src& s, int64_t row, int width, int col) {
    float f[8];
    if (s.lm_rows > 0) {  // feature pairs col/2 .. col/2+3 of the row, one per level plane
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t e = ((int64_t)(col / 2 + q) * s.lm_rows + row) * 2;
            if (s.dtype == AVR_DTYPE_F16) {
                const float2 v = __half22float2(*reinterpret_cast<const __half2*>(static_cast<const __half*>(s.p) + e));
                f[2 * q] = v.x;
                f[2 * q + 1] = v.y;
            } else {
                const float2 v = *reinterpret_cast<const float2*>(static_cast<const float*>(s.p) + e);
                f[2 * q] = v.x;
                f[2 * q + 1] = v.y;
            }
        }
    } else if (s.dtype == AVR_DTYPE_F16) {
        const u32x4v v = *reinterpret_cast<const u32x4v*>(
            static_cast<const __half*>(s.p) + row * width + col);
        Vec16<__half>::cvt(v, f);
    } else {
        const float* q = static_cast<const float*>(s.p) + row * width + col;
        const f32x4 a = *reinterpret_cast<const f32x4*>(q);
        const f32x4 b = *reinterpret_cast<const f32x4*>(q + 4);
        f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
        f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
    }
    frag8 r;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = pack2<E>(f[2 * q], f[2 * q + 1]);
    return r;
}

// Cooperative global -> LDS staging of 32 KB chunks into two LDS buffers.
// Chunk c is read from buffer c & 1; while it is computed, chunk c+1 sits in
// registers (its loads were issued a whole chunk earlier).  After computing
// chunk c each wave writes its share of chunk c+1 into the other buffer (whose
// last readers, chunk c-1, all passed the previous barrier), then ONE raw
// barrier (LDS writes drained, outstanding global stores NOT waited for),
// then the loads of chunk c+2 are issued.
// DBG (timing experiments only, tools/probe_sigma.py tile_cfg >= 16): bit 0
// drops the barrier, bit 1 the staging loads/writes (results are garbage).
// Bits 32 and 64 are not experiments but staging modes (the h1 kernel's
// default uses both, tile_cfg 0; 2-4% faster than register staging).
// DMA (DBG bit 32): the chunks travel global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, issued as inline asm: the compiler does not
// track it, so it neither waits on it inside the MFMA chains nor treats it
// as an LDS write), no staging registers and no ds_write.  Chunk c+2 is
// issued into buffer c & 1 right after the barrier that ends chunk c; the
// barrier before chunk c+1 first waits for this wave's DMA (vmcnt(0): the
// previous chunk's h1 stores, issued after the DMA of chunk c+1, have had a
// whole chunk of MFMAs to drain).
template <int WAVES, int DBG = 0>
struct Stager {
    static constexpr bool kDma = (DBG & 32) != 0;
    static constexpr int kPer = kChunk / (64 * WAVES * 16);
    u32x4v r[kDma ? 1 : kPer];
    const u32x4v* src;
    char* lds;
    int cur, n_chunks, tid;
    bool defer = false;  // DMA mode: finish_chunk leaves the next issue to issue_deferred()
    int pending = -1;
    __device__ void issue_deferred() {
        if (pending >= 0) issue(pending);
        pending = -1;
    }
    __device__ void issue(int c) {
        const u32x4v* p = src + (int64_t)c * (kChunk / 16);
        if constexpr (kDma) {
            const uint32_t base = (uint32_t)(uintptr_t)(lds + (c & 1) * kChunk) + (tid & ~63) * 16;
#pragma unroll
            for (int i = 0; i < kPer; ++i) {
                const uint32_t m = __builtin_amdgcn_readfirstlane(base + 64 * WAVES * 16 * i);
                asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                             ::"s"(m), "v"(p + tid + 64 * WAVES * i) : "memory", "m0");
            }
        } else {
#pragma unroll
            for (int i = 0; i < kPer; ++i) r[i] = p[tid + 64 * WAVES * i];
        }
    }
    __device__ void write(int c) {
        if constexpr (!kDma) {
            u32x4v* d = reinterpret_cast<u32x4v*>(lds + (c & 1) * kChunk);
#pragma unroll
            for (int i = 0; i < kPer; ++i) d[tid + 64 * WAVES * i] = r[i];
        }
    }
    __device__ static void barrier() {
        if constexpr (kDma)
            asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    __device__ void start(const char* wpack, char* lds_base, int chunks) {
        src = reinterpret_cast<const u32x4v*>(wpack);
        lds = lds_base;
        tid = threadIdx.x;
        n_chunks = chunks;
        cur = 0;
        if constexpr (kDma) {
            issue(0);
            if (chunks > 1) issue(1);
        } else {
            issue(0);
            write(0);
            if (chunks > 1) issue(1);
        }
        barrier();
    }
    __device__ const char* buffer() const { return lds + (cur & 1) * kChunk; }
    __device__ void finish_chunk() {
        if constexpr (kDma) {
            barrier();  // this wave's DMA of chunk cur+1 landed; every wave left buffer cur & 1
            if (cur + 2 < n_chunks) {
                if (defer)
                    pending = cur + 2;
                else
                    issue(cur + 2);
            }
        } else {
            if constexpr (!(DBG & 2)) {
                if (cur + 1 < n_chunks) write(cur + 1);
            }
            if constexpr (!(DBG & 1)) barrier();
            if constexpr (!(DBG & 2)) {
                if (cur + 2 < n_chunks) issue(cur + 2);
            }
        }
        ++cur;
    }
};

// The layer's B operands stay in their registers until every MFMA of the
// layer has issued and the queue wait has passed (common.h): the next
// layer's fragments, weight reads and accumulators are not allocated onto
// them while one of the layer's MFMAs may still wait to read them.
template <int NT, int KS>
__device__ __forceinline__ void hold_operands(const frag8 (&x)[NT][KS]) {
    mfma_queue_wait();
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) keep_live(x[nt][ks]);
}

// acc[nt][ot] = W X^T for one layer: KS k-steps of input fragments, OT output
// tiles, CO tiles per LDS chunk.  ZERO = false: acc holds the start values
// (the h1 layer's bias) and the products are accumulated onto them.
template <typename E, int NT, int KS, int OT, int CO, class ST, bool ZERO = true>
__device__ __forceinline__ void dense(ST& st, int lane,
                                      const frag8 (&x)[NT][KS], f32x16 (&acc)[NT][OT]) {
    static_assert(OT % CO == 0 && CO * KS * kFrag <= kChunk, "chunk overflow");
    if constexpr (ZERO) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int ot = 0; ot < OT; ++ot)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[nt][ot][i] = 0.0f;
    }
#pragma unroll
    for (int c = 0; c < OT / CO; ++c) {
        const char* lds = st.buffer();
        // k-step outer: the CO*NT accumulators of a k-step are independent,
        // so no MFMA waits on the previous one's result; the next k-step's
        // CO weight fragments are read while this one's MFMAs run
        frag8 a[2][CO];
#pragma unroll
        for (int o = 0; o < CO; ++o)
            a[0][o] = *reinterpret_cast<const frag8*>(lds + (o * KS) * kFrag + lane * 16);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (ks + 1 < KS) {
#pragma unroll
                for (int o = 0; o < CO; ++o)
                    a[(ks + 1) & 1][o] =
                        *reinterpret_cast<const frag8*>(lds + (o * KS + ks + 1) * kFrag + lane * 16);
            }
#pragma unroll
            for (int o = 0; o < CO; ++o)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[nt][c * CO + o] = mfma16<E>(a[ks & 1][o], x[nt][ks], acc[nt][c * CO + o]);
        }
        st.finish_chunk();
    }
    hold_operands(x);
}

// one accumulator tile -> 8 dwords of E: dword q holds registers 2q, 2q+1
template <typename E>
__device__ __forceinline__ void pack_tile(const f32x16& acc, uint32_t (&d)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = pack2<E>(acc[2 * q], acc[2 * q + 1]);
}

// packed tile -> next layer's B fragments (k-step 2*ot + s = registers 8s..8s+7)
__device__ __forceinline__ void tile_frags(const uint32_t (&d)[8], bool rectify, frag8& x0, frag8& x1) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        x0[q] = rectify ? relu16x2(d[q]) : d[q];
        x1[q] = rectify ? relu16x2(d[4 + q]) : d[4 + q];
    }
}

template <typename E, int NT, int OT>
__device__ __forceinline__ void to_frags(const f32x16 (&acc)[NT][OT], frag8 (&x)[NT][2 * OT]) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int ot = 0; ot < OT; ++ot) {
            uint32_t d[8];
            pack_tile<E>(acc[nt][ot], d);
            tile_frags(d, true, x[nt][2 * ot], x[nt][2 * ot + 1]);
        }
}

// store OT output tiles (bf16, optionally rectified) into base columns
// [0, 32*OT) and return them as the next layer's (rectified) fragments: lane
// (column n, half h) holds rows 8g + 4h + 0..3 of each tile in registers
// 4g..4g+3 -> one 8-byte store per g.
template <typename E, int NT, int OT>
__device__ __forceinline__ void store_and_frags(const Args& a, const f32x16 (&acc)[NT][OT], int64_t n0,
                                                int lane, bool rectify, frag8 (&x)[NT][2 * OT]) {
    const int h = lane >> 5;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int64_t n = n0 + 32 * nt + (lane & 31);
        uint16_t* row = a.base + n * a.ldb;
#pragma unroll
        for (int ot = 0; ot < OT; ++ot) {
            uint32_t d[8];
            pack_tile<E>(acc[nt][ot], d);
            if (rectify) {
#pragma unroll
                for (int q = 0; q < 8; ++q) d[q] = relu16x2(d[q]);
            }
            if (n < a.N) {
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *reinterpret_cast<u32x2v*>(row + 32 * ot + 8 * g + 4 * h) = u32x2v{d[2 * g], d[2 * g + 1]};
            }
            tile_frags(d, !rectify, x[nt][2 * ot], x[nt][2 * ot + 1]);
        }
    }
}

// decoder output (row 0 of the single output tile: register 0 of lanes 0..31)
template <typename E, int NT>
__device__ __forceinline__ void store_attn(const Args& a, const f32x16 (&acc)[NT][1], int64_t n0, int lane) {
    if (lane >= 32) return;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int64_t n = n0 + 32 * nt + lane;
        if (n >= a.N) continue;
        const float y = round16<E>(acc[nt][0][0]);       // the GEMM's 16-bit output
        const float l = y > 0.0f ? y : y * a.slope;      // leaky_relu in fp32 ...
        const float r = fabsf(round16<E>(l));            // ... rounded to E, abs
        a.attn[n] = bits16<E>(r);
    }
}

// row of source s that sample n reads (32-bit: N < 2^31 is checked on the host)
__device__ __forceinline__ int64_t src_row(const Src& s, int64_t n) {
    return (int64_t)((uint32_t)n / (uint32_t)s.rows_div);
}

// extra feature segments copied (as bf16) into base columns after the MLP
// output: lane (sample r, half h) copies 8-feature chunks h, h+2, ... of its
// sample's row of every segment (one division per segment and lane)
template <typename E, int NT>
__device__ __forceinline__ void copy_extras(const Args& a, int64_t n0, int lane) {
    const int h = lane >> 5;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int64_t n = n0 + 32 * nt + (lane & 31);
        if (n >= a.N) continue;
        uint16_t* row = a.base + n * a.ldb;
        for (int e = 0; e < a.n_extra; ++e) {
            const Src s = a.extra[e];
            const int w = a.extra_width[e];
            const int64_t r = src_row(s, n);
            for (int c = 8 * h; c < w; c += 16)
                *reinterpret_cast<frag8*>(row + a.extra_col[e] + c) = load8<E>(s, r, w, c);
        }
    }
}

// first-layer input fragments: lane (sample r, half h) k-step ks holds
// features 8c..8c+7 with c = 2ks + h; chunks [0, 5) come from in0 (40 per
// sample), [5, 10) from in1 (40 per pose) when the net has two inputs.
template <typename E, int NT, int KS0>
__device__ __forceinline__ void load_input(const Args& a, int64_t n0, int lane, frag8 (&x)[NT][KS0]) {
    const int h = lane >> 5;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        int64_t n = n0 + 32 * nt + (lane & 31);
        n = n < a.N ? n : a.N - 1;
        const int64_t r0 = src_row(a.in0, n);
        const int64_t r1 = KS0 > 3 ? src_row(a.in1, n) : 0;
#pragma unroll
        for (int ks = 0; ks < KS0; ++ks) {
            const int c = 2 * ks + h;
            if (c < 5) {
                x[nt][ks] = load8<E>(a.in0, r0, 40, 8 * c);
            } else if (KS0 > 3 && c < 10) {
                x[nt][ks] = load8<E>(a.in1, r1, 40, 8 * (c - 5));
            } else {
                x[nt][ks] = frag8{0u, 0u, 0u, 0u};  // +0 in either format
            }
        }
    }
}

// Variant 0 (AVRModel): 40 -> 128 -> 128 -> 128 -> 128 (linear, = sigma_feat)
// -> relu -> 128 -> 128 -> 128 -> 1.  8 chunks.
template <typename E, int NT, int WAVES, int OCC, int DBG = 0>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(OCC)))
void sigma_meshrir_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kChunk];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t n0 = ((int64_t)blockIdx.x * WAVES + wave) * 32 * NT;
    Stager<WAVES, DBG> st;
    st.start(a.wpack, lds, 8);

    frag8 x0[NT][3];
    load_input<E, NT, 3>(a, n0, lane, x0);
    frag8 x[NT][8];
    {
        f32x16 acc[NT][4];
        dense<E, NT, 3, 4, 4>(st, lane, x0, acc);
        to_frags<E, NT, 4>(acc, x);
    }
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        f32x16 acc[NT][4];
        dense<E, NT, 8, 4, 4>(st, lane, x, acc);
        to_frags<E, NT, 4>(acc, x);
    }
    {
        f32x16 acc[NT][4];
        dense<E, NT, 8, 4, 4>(st, lane, x, acc);
        // sigma_feat (linear) -> base; relu(sigma_feat) -> decoder
        store_and_frags<E, NT, 4>(a, acc, n0, lane, false, x);
    }
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        f32x16 acc[NT][4];
        dense<E, NT, 8, 4, 4>(st, lane, x, acc);
        to_frags<E, NT, 4>(acc, x);
    }
    {
        f32x16 acc[NT][1];
        dense<E, NT, 8, 1, 1>(st, lane, x, acc);
        store_attn<E, NT>(a, acc, n0, lane);
    }
    if constexpr (!(DBG & 4)) copy_extras<E, NT>(a, n0, lane);
}

// the h1 layer's accumulators start at the bias: acc[nt][ot] register 4g + e
// = bias[n / bias_div][128 c + 32 ot + 8 g + 4 h + e] of the lane's sample n
// (the per-ray / per-pose columns' part of the layer, summed before the
// per-sample products instead of after them: one fp32 sum order of the
// same terms, and 16 fewer VALU adds per tile)
template <int NT>
__device__ __forceinline__ void bias_acc(const Args& a, f32x16 (&acc)[NT][4], int64_t n0, int lane, int c) {
    const int h = lane >> 5, r = lane & 31;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int64_t n = n0 + 32 * nt + r;
        const int64_t nl = n < a.N ? n : a.N - 1;
        const float* brow = a.bias + (int64_t)((uint32_t)nl / (uint32_t)a.bias_div) * 512 + 128 * c;
#pragma unroll
        for (int ot = 0; ot < 4; ++ot)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 b = *reinterpret_cast<const f32x4*>(brow + 32 * ot + 8 * g + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[nt][ot][4 * g + e] = b[e];
            }
    }
}

// signal layer 1 epilogue (variant 2): h1[n][128c + o] = bf16(relu(acc)), acc
// started at bias[n / bias_div][128c + o] (bias_acc).
// The MFMA result has the sample on the lane, so written straight out every
// store instruction would touch 32 rows x 16 B; instead each pair of tiles
// (32 samples x 64 columns, 4 KB) goes through a per-wave LDS area (16-byte
// chunks XOR-swizzled by row: conflict-free) and leaves as 4 instructions
// of 8 rows x 128 contiguous bytes (full cache lines).
template <typename E, int NT, bool STORE = true>
__device__ __forceinline__ void store_h1(const Args& a, const f32x16 (&acc)[NT][4], int64_t n0, int lane, int c,
                                         char* tr) {
    const int h = lane >> 5, r = lane & 31;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int ot = 2 * p + j;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x16& v = acc[nt][ot];
                    const uint32_t w0 = pack2<E>(relu(v[4 * g]), relu(v[4 * g + 1]));
                    const uint32_t w1 = pack2<E>(relu(v[4 * g + 2]), relu(v[4 * g + 3]));
                    const int ch = (4 * j + g) ^ (r & 7);  // 16-B chunk of the 128-B row
                    *reinterpret_cast<u32x2v*>(tr + r * 128 + ch * 16 + 8 * h) = u32x2v{w0, w1};
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 8 * q + (lane >> 3), chunk = lane & 7;
                const u32x4v v = *reinterpret_cast<const u32x4v*>(tr + row * 128 + ((chunk ^ (row & 7)) * 16));
                const int64_t nr = n0 + 32 * nt + row;
                // (STORE = false: timing experiments; a.ldb < 0 never holds)
                if (STORE ? nr < a.N : a.ldb < 0) {
                    u32x4v* dst = reinterpret_cast<u32x4v*>(a.base + nr * a.ldb + 128 * c + 64 * p + 8 * chunk);
                    if (a.nt_store)
                        __builtin_nontemporal_store(v, dst);
                    else
                        *dst = v;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
}

// Variant 2 (AVRModel, sigma networks + the signal network's first layer):
// the sigma encoder, then h1 = relu(W1[:, :128] sigma_feat + bias[ray]) with
// the per-ray / per-pose columns of the layer (dir_enc, tx_enc) folded into
// `bias` on the host, written as [N][512] bf16 in place of the concatenated
// input, then the decoder on relu(sigma_feat).  12 chunks, in that order
// (sigma.py STREAM_ORDER): the h1 layer runs while bf16(sigma_feat) is the
// only live activation, and the decoder's input is rectified from it in
// place, so one copy of the features is held instead of two (32 VGPRs per
// 32-sample tile).
template <typename E, int NT, int WAVES, int OCC, int DBG = 0>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(OCC)))
void sigma_meshrir_h1_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kChunk + WAVES * 4096];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t n0 = ((int64_t)blockIdx.x * WAVES + wave) * 32 * NT;
    Stager<WAVES, DBG & 99> st;
    st.start(a.wpack, lds, 12);
    using ST = decltype(st);

    frag8 x0[NT][3];
    load_input<E, NT, 3>(a, n0, lane, x0);
    frag8 x[NT][8];
    {
        f32x16 acc[NT][4];
        dense<E, NT, 3, 4, 4>(st, lane, x0, acc);
        to_frags<E, NT, 4>(acc, x);
    }
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        f32x16 acc[NT][4];
        dense<E, NT, 8, 4, 4>(st, lane, x, acc);
        to_frags<E, NT, 4>(acc, x);
    }
    {
        // x <- bf16(sigma_feat) (linear): the signal network's per-sample input
        f32x16 acc[NT][4];
        dense<E, NT, 8, 4, 4>(st, lane, x, acc);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int ot = 0; ot < 4; ++ot) {
                uint32_t d[8];
                pack_tile<E>(acc[nt][ot], d);
                tile_frags(d, false, x[nt][2 * ot], x[nt][2 * ot + 1]);
            }
    }
    // DBG & 64 (with the DMA stager): each h1 chunk's weight DMA is issued
    // after the previous chunk's epilogue, whose bias loads would otherwise
    // wait for it (vmcnt counts in order)
    if constexpr ((DBG & 64) != 0) st.defer = true;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        f32x16 acc[NT][4];
        bias_acc<NT>(a, acc, n0, lane, c);
        dense<E, NT, 8, 4, 4, ST, false>(st, lane, x, acc);
        store_h1<E, NT, !(DBG & 4)>(a, acc, n0, lane, c, lds + 2 * kChunk + wave * 4096);
        if constexpr ((DBG & 64) != 0) st.issue_deferred();
    }
    st.defer = false;
    // the decoder's input: relu(sigma_feat), rectified in the 16-bit format
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) x[nt][k][q] = relu16x2(x[nt][k][q]);
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        f32x16 acc[NT][4];
        dense<E, NT, 8, 4, 4>(st, lane, x, acc);
        to_frags<E, NT, 4>(acc, x);
    }
    {
        f32x16 acc[NT][1];
        dense<E, NT, 8, 1, 1>(st, lane, x, acc);
        store_attn<E, NT>(a, acc, n0, lane);
    }
}

// Variant 1 (AVRModel_complex): [40 | 40] -> 128 -> 128 -> 128 -> 256 (relu,
// = rf) -> 128 -> 1.  8 chunks (the 256-wide layers take two each).
template <typename E, int NT, int WAVES, int OCC>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(OCC)))
void sigma_raf_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) char lds[2 * kChunk];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t n0 = ((int64_t)blockIdx.x * WAVES + wave) * 32 * NT;
    Stager<WAVES> st;
    st.start(a.wpack, lds, 8);

    frag8 x0[NT][5];
    load_input<E, NT, 5>(a, n0, lane, x0);
    frag8 x[NT][8];
    {
        f32x16 acc[NT][4];
        dense<E, NT, 5, 4, 4>(st, lane, x0, acc);
        to_frags<E, NT, 4>(acc, x);
    }
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        f32x16 acc[NT][4];
        dense<E, NT, 8, 4, 4>(st, lane, x, acc);
        to_frags<E, NT, 4>(acc, x);
    }
    frag8 rf[NT][16];
    {
        f32x16 acc[NT][8];
        dense<E, NT, 8, 8, 4>(st, lane, x, acc);
        store_and_frags<E, NT, 8>(a, acc, n0, lane, true, rf);  // rf = relu(sigma_feature)
    }
    {
        f32x16 acc[NT][4];
        dense<E, NT, 16, 4, 2>(st, lane, rf, acc);
        to_frags<E, NT, 4>(acc, x);
    }
    {
        f32x16 acc[NT][1];
        dense<E, NT, 8, 1, 1>(st, lane, x, acc);
        store_attn<E, NT>(a, acc, n0, lane);
    }
    copy_extras<E, NT>(a, n0, lane);
}

bool src_ok(const avr_feat_src& s) {
    return s.data && (s.dtype == AVR_DTYPE_F16 || s.dtype == AVR_DTYPE_F32) && s.rows_div >= 1 &&
           s.lm_rows >= 0 && reinterpret_cast<uintptr_t>(s.data) % 16 == 0;
}

Src to_src(const avr_feat_src& s) { return Src{s.data, (int)s.dtype, (int)s.rows_div, s.lm_rows}; }

template <typename E, int NT, int WAVES, int OCC, int DBG = 0>
int launch_meshrir(const Args& a, hipStream_t st) {
    const int64_t per_block = 32 * NT * WAVES;
    const dim3 grid((unsigned)((a.N + per_block - 1) / per_block));
    hipLaunchKernelGGL((sigma_meshrir_kernel<E, NT, WAVES, OCC, DBG>), grid, dim3(64 * WAVES), 0, st, a);
    return check_launch("avr_sigma_fwd");
}

template <typename E, int NT, int WAVES, int OCC, int DBG = 0>
int launch_meshrir_h1(const Args& a, hipStream_t st) {
    const int64_t per_block = 32 * NT * WAVES;
    const dim3 grid((unsigned)((a.N + per_block - 1) / per_block));
    hipLaunchKernelGGL((sigma_meshrir_h1_kernel<E, NT, WAVES, OCC, DBG>), grid, dim3(64 * WAVES), 0, st, a);
    return check_launch("avr_sigma_fwd");
}

template <typename E, int WAVES, int OCC>
int launch_raf(const Args& a, hipStream_t st) {
    const int64_t per_block = 32 * WAVES;
    const dim3 grid((unsigned)((a.N + per_block - 1) / per_block));
    hipLaunchKernelGGL((sigma_raf_kernel<E, 1, WAVES, OCC>), grid, dim3(64 * WAVES), 0, st, a);
    return check_launch("avr_sigma_fwd");
}

}  // namespace

namespace {
template <typename E>
int dispatch(const avr_sigma_desc* d, Args& a, bool h1, bool two, hipStream_t st);
}

extern "C" int avr_sigma_pack_bytes(int32_t variant, int64_t* bytes) {
    AVR_REQUIRE(bytes && (variant == AVR_SIGMA_MESHRIR || variant == AVR_SIGMA_RAF ||
                          variant == AVR_SIGMA_MESHRIR_H1),
                "avr_sigma_pack_bytes: bad variant");
    *bytes = (variant == AVR_SIGMA_MESHRIR_H1 ? 12 : 8) * (int64_t)kChunk;
    return 0;
}

extern "C" int avr_sigma_fwd(const avr_sigma_desc* d, const void* wpack, void* base, int32_t ldb,
                             void* attn, void* stream) {
    AVR_REQUIRE(d && wpack && base && attn, "avr_sigma_fwd: null argument");
    AVR_REQUIRE(d->variant == AVR_SIGMA_MESHRIR || d->variant == AVR_SIGMA_RAF ||
                    d->variant == AVR_SIGMA_MESHRIR_H1,
                "avr_sigma_fwd: bad variant");
    const bool h1 = d->variant == AVR_SIGMA_MESHRIR_H1;
    AVR_REQUIRE(!h1 || (d->bias && d->bias_div >= 1 && ldb == 512 && d->n_extra == 0 &&
                        reinterpret_cast<uintptr_t>(d->bias) % 16 == 0),
                "avr_sigma_fwd: variant MESHRIR_H1 needs bias, bias_div >= 1, ldb 512, no extras");
    AVR_REQUIRE(d->n_samples >= 1 && d->n_samples < (int64_t(1) << 31),
                "avr_sigma_fwd: n_samples must be in [1, 2^31)");
    const bool two = d->variant == AVR_SIGMA_RAF;
    AVR_REQUIRE(src_ok(d->input[0]) && (!two || src_ok(d->input[1])), "avr_sigma_fwd: bad input source");
    AVR_REQUIRE(d->n_extra >= 0 && d->n_extra <= AVR_SIGMA_MAX_EXTRA, "avr_sigma_fwd: bad n_extra");
#if defined(AVR_PHASE_PROBES) || defined(AVR_SHAPE_PROBES)
    AVR_REQUIRE(d->tile_cfg >= 0 && d->tile_cfg <= 20, "avr_sigma_fwd: bad tile_cfg");
#else
    // 0..8 are tilings with correct results; the timing experiments (16..20)
    // exist only in the probe builds
    AVR_REQUIRE(d->tile_cfg >= 0 && d->tile_cfg <= 8, "avr_sigma_fwd: bad tile_cfg");
#endif
    const int out_w = two ? 256 : (d->variant == AVR_SIGMA_MESHRIR_H1 ? 512 : 128);
    AVR_REQUIRE(ldb % 8 == 0 && reinterpret_cast<uintptr_t>(base) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(wpack) % 16 == 0,
                "avr_sigma_fwd: base/wpack must be 16-byte aligned, ldb a multiple of 8");
    Args a{};
    a.N = d->n_samples;
    a.in0 = to_src(d->input[0]);
    a.in1 = two ? to_src(d->input[1]) : a.in0;
    a.n_extra = d->n_extra;
    int col = out_w;
    for (int e = 0; e < d->n_extra; ++e) {
        AVR_REQUIRE(src_ok(d->extra[e]) && d->extra_width[e] >= 8 && d->extra_width[e] % 8 == 0,
                    "avr_sigma_fwd: bad extra feature source");
        a.extra[e] = to_src(d->extra[e]);
        a.extra_width[e] = d->extra_width[e];
        a.extra_col[e] = col;
        col += d->extra_width[e];
    }
    AVR_REQUIRE(col <= ldb, "avr_sigma_fwd: ldb smaller than the concatenated features");
    a.wpack = static_cast<const char*>(wpack);
    a.base = static_cast<uint16_t*>(base);
    a.ldb = ldb;
    a.attn = static_cast<uint16_t*>(attn);
    a.slope = d->leaky_slope;
    a.bias = d->bias;
    a.bias_div = d->bias_div;
    AVR_REQUIRE(d->dtype == AVR_DTYPE_BF16 || d->dtype == AVR_DTYPE_F16,
                "avr_sigma_fwd: dtype must be AVR_DTYPE_BF16 or AVR_DTYPE_F16");
    hipStream_t st = as_stream(stream);
    if (d->dtype == AVR_DTYPE_F16) return dispatch<_Float16>(d, a, h1, two, st);
    return dispatch<__bf16>(d, a, h1, two, st);
}

namespace {
template <typename E>
int dispatch(const avr_sigma_desc* d, Args& a, bool h1, bool two, hipStream_t st) {
    if (h1) {
        // 0: 4 waves, streaming h1 stores (120 us at config 2); 1: 8 waves;
        // 2, 3: the same with plain stores (130 us)
        a.nt_store = d->tile_cfg < 2;
        if (const char* f = AVR_PROBE_ENV("AVR_SIGMA_NT_PROBE")) a.nt_store = f[0] == '1';  // shapes build only
        if (d->tile_cfg == 1 || d->tile_cfg == 3) return launch_meshrir_h1<E, 1, 8, 1>(a, st);
        // 4, 5: 64 samples per wave (each weight fragment feeds two MFMAs),
        // 1 or 2 waves per SIMD (experiments)
        if (d->tile_cfg == 4) return launch_meshrir_h1<E, 2, 4, 1>(a, st);
        if (d->tile_cfg == 6) return launch_meshrir_h1<E, 1, 4, 2, 32>(a, st);  // LDS-DMA weight staging
        if (d->tile_cfg == 7) return launch_meshrir_h1<E, 1, 4, 2, 96>(a, st);  // + h1 DMAs after the epilogue
        if (d->tile_cfg == 5) return launch_meshrir_h1<E, 2, 4, 2>(a, st);
#if defined(AVR_PHASE_PROBES) || defined(AVR_SHAPE_PROBES)
        // timing experiments (results are garbage; probe builds only): no
        // barrier / no weight staging / no h1 stores (bf16 only)
        if constexpr (std::is_same<E, __bf16>::value) {
            if (d->tile_cfg == 16) return launch_meshrir_h1<E, 1, 4, 2, 1>(a, st);
            if (d->tile_cfg == 17) return launch_meshrir_h1<E, 1, 4, 2, 2>(a, st);
            if (d->tile_cfg == 18) return launch_meshrir_h1<E, 1, 4, 2, 4>(a, st);
            if (d->tile_cfg == 19) return launch_meshrir_h1<E, 1, 4, 2, 7>(a, st);
        }
#endif
        if (d->tile_cfg == 8) return launch_meshrir_h1<E, 1, 4, 2>(a, st);  // register-staged weights
        return launch_meshrir_h1<E, 1, 4, 2, 96>(a, st);  // LDS-DMA staging, h1 DMAs after the epilogue
    }
    const int cfg = d->tile_cfg;
    // tile configs (tools/probe_sigma.py, MI355X at config 2, fp16;
    // profiles/r06_sigma_tilings.jsonl): MeshRIR 0 = 32 samples per wave, 4
    // waves at 2 waves/SIMD (73.7 us, no scratch); 1 = 32 per wave, 8 waves
    // (75.4 us); 2 = 64 per wave, 4 waves, 2 waves/SIMD (80.3 us: 68 bytes of
    // scratch per lane once the layer's B operands are held, §15a; the default
    // until round 5); 3 = 64 per wave, 4 waves, 1 wave/SIMD (92.7 us).
    // RAF: 0 = 4 waves (120 us), 1 = 8 waves (137 us).
    if (two) return cfg == 1 ? launch_raf<E, 8, 1>(a, st) : launch_raf<E, 4, 2>(a, st);
    if (cfg == 1) return launch_meshrir<E, 1, 8, 1>(a, st);
    if (cfg == 2) return launch_meshrir<E, 2, 4, 2>(a, st);
    if (cfg == 3) return launch_meshrir<E, 2, 4, 1>(a, st);
#if defined(AVR_PHASE_PROBES) || defined(AVR_SHAPE_PROBES)
    if constexpr (std::is_same<E, __bf16>::value) {  // timing experiments, garbage results
        if (cfg == 16) return launch_meshrir<E, 1, 8, 1, 1>(a, st);
        if (cfg == 17) return launch_meshrir<E, 1, 8, 1, 2>(a, st);
        if (cfg == 18) return launch_meshrir<E, 1, 8, 1, 3>(a, st);
        if (cfg == 19) return launch_meshrir<E, 1, 8, 1, 4>(a, st);
        if (cfg == 20) return launch_meshrir<E, 1, 8, 1, 7>(a, st);
    }
#endif
    return launch_meshrir<E, 1, 4, 2>(a, st);
}
}  // namespace

extern "C" int avr_sigma_desc_size(void) { return (int)sizeof(avr_sigma_desc); }
