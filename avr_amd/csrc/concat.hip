// Grouped feature concatenation for the networks' training path and its
// adjoint (a6: the inputs of the sigma encoder and of the signal network,
// model.py:199-221 / 314-325).
//
//   out[n][col_i + c] = cast(src_i[n / rows_div_i][c])       (forward)
//   grad_i[r][c] = sum_{n: n / rows_div_i = r} grad_out[n][col_i + c]   (backward)
//
// A source is per sample (rows_div 1), per ray (S) or per pose (R*S): the
// per-ray / per-pose encodings are evaluated once per group and read here by
// every sample of the group, instead of being expanded to [N, 40] copies and
// concatenated (two passes over the output), and their gradient is summed
// over the group in fp32 with a fixed order (deterministic) instead of a
// strided torch reduction per source.
#include "common.h"

using namespace avr;

namespace {

constexpr int kMaxSrc = AVR_CONCAT_MAX_SRC;
constexpr int kMaxChunks = 64;  // output width <= 512

struct Table {
    const void* p[kMaxSrc];
    int dtype[kMaxSrc];
    int rows_div[kMaxSrc];
    int width[kMaxSrc];
    unsigned char chunk_src[kMaxChunks];
    short chunk_off[kMaxChunks];
};

__device__ __forceinline__ void load8(const void* base, int dtype, int64_t e, float* f) {
    if (dtype == AVR_DTYPE_F32) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + e);
        const f32x4 b = *reinterpret_cast<const f32x4*>(static_cast<const float*>(base) + e + 4);
        f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
        f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
    } else {
        const u32x4 v = *reinterpret_cast<const u32x4*>(static_cast<const uint16_t*>(base) + e);
        if (dtype == AVR_DTYPE_F16) {
            Vec16<__half>::cvt(v, f);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                f[2 * i] = bf16_lo(v[i]);
                f[2 * i + 1] = bf16_hi(v[i]);
            }
        }
    }
}

__device__ __forceinline__ void store8(void* base, int dtype, int64_t e, const float* f) {
    if (dtype == AVR_DTYPE_F32) {
        float* q = static_cast<float*>(base) + e;
        *reinterpret_cast<f32x4*>(q) = f32x4{f[0], f[1], f[2], f[3]};
        *reinterpret_cast<f32x4*>(q + 4) = f32x4{f[4], f[5], f[6], f[7]};
    } else if (dtype == AVR_DTYPE_F16) {
        u32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const __half2 h = __floats2half2_rn(f[2 * i], f[2 * i + 1]);
            v[i] = *reinterpret_cast<const uint32_t*>(&h);
        }
        *reinterpret_cast<u32x4*>(static_cast<uint16_t*>(base) + e) = v;
    } else {
        u32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const __hip_bfloat16 a = __float2bfloat16(f[2 * i]), b = __float2bfloat16(f[2 * i + 1]);
            v[i] = (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
        }
        *reinterpret_cast<u32x4*>(static_cast<uint16_t*>(base) + e) = v;
    }
}

// one thread per (row, 8-column chunk); consecutive threads = consecutive
// chunks of a row (coalesced stores)
__global__ __launch_bounds__(256) void concat_fwd_kernel(uint32_t N, int nch, Table t, void* out,
                                                         int out_dtype) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= N * (uint32_t)nch) return;
    const uint32_t n = q / (uint32_t)nch;
    const int c = (int)(q - n * (uint32_t)nch);
    const int s = t.chunk_src[c];
    const uint32_t row = n / (uint32_t)t.rows_div[s];
    float f[8];
    load8(t.p[s], t.dtype[s], (int64_t)row * t.width[s] + t.chunk_off[c], f);
    store8(out, out_dtype, (int64_t)q * 8, f);
}

// dst[r][8c .. 8c+7] = sum over the div rows of group r of g[n*ldg + col + 8c ..]:
// J lanes per (r, c), lane j takes rows j, j+J, ...; fixed xor tree over the
// J lanes (deterministic).
template <int J>
__global__ __launch_bounds__(256) void group_sum_kernel(uint32_t n_out, int div, int w8,
                                                        const void* g, int g_dtype, int64_t ldg, int col,
                                                        void* dst, int dst_dtype) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    const uint32_t item = t / J;
    const int j = (int)(t % J);
    const bool live = item < n_out * (uint32_t)w8;
    const uint32_t r = live ? item / (uint32_t)w8 : 0;
    const int c = live ? (int)(item - r * (uint32_t)w8) : 0;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (live) {
        const int64_t n0 = (int64_t)r * div;
        for (int k = j; k < div; k += J) {
            float f[8];
            load8(g, g_dtype, (n0 + k) * ldg + col + 8 * c, f);
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] += f[i];
        }
    }
#pragma unroll
    for (int off = J / 2; off > 0; off >>= 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += __shfl_xor(acc[i], off, 64);
    }
    if (live && j == 0) store8(dst, dst_dtype, (int64_t)r * (8 * w8) + 8 * c, acc);
}

bool dtype_ok(int d) { return d == AVR_DTYPE_F32 || d == AVR_DTYPE_F16 || d == AVR_DTYPE_BF16; }

int launch_group_sum(uint32_t n_out, int div, int w8, const void* g, int g_dtype, int64_t ldg, int col,
                     void* dst, int dst_dtype, hipStream_t st) {
    const uint64_t items = (uint64_t)n_out * w8;
    auto go = [&](auto kern, int J) {
        const uint64_t threads = items * J;
        hipLaunchKernelGGL(kern, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, n_out, div, w8, g,
                           g_dtype, ldg, col, dst, dst_dtype);
    };
    if (div == 1)
        go(group_sum_kernel<1>, 1);
    else if (div <= 64)
        go(group_sum_kernel<8>, 8);
    else
        go(group_sum_kernel<64>, 64);
    return check_launch("avr_concat_bwd");
}

}  // namespace

extern "C" int avr_concat_fwd(int64_t N, int32_t n_src, const avr_concat_src* src, void* out,
                              int32_t out_dtype, void* stream) {
    AVR_REQUIRE(src && out && n_src >= 1 && n_src <= kMaxSrc && dtype_ok(out_dtype),
                "avr_concat_fwd: bad arguments");
    Table t{};
    int col = 0;
    for (int i = 0; i < n_src; ++i) {
        const avr_concat_src& s = src[i];
        AVR_REQUIRE(s.data && dtype_ok(s.dtype) && s.rows_div >= 1 && s.width >= 8 && s.width % 8 == 0 &&
                        reinterpret_cast<uintptr_t>(s.data) % 16 == 0,
                    "avr_concat_fwd: bad source");
        t.p[i] = s.data;
        t.dtype[i] = s.dtype;
        t.rows_div[i] = s.rows_div;
        t.width[i] = s.width;
        for (int c = 0; c < s.width / 8; ++c) {
            AVR_REQUIRE(col / 8 < kMaxChunks, "avr_concat_fwd: output wider than 512");
            t.chunk_src[col / 8] = (unsigned char)i;
            t.chunk_off[col / 8] = (short)(8 * c);
            col += 8;
        }
    }
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(out) % 16 == 0, "avr_concat_fwd: out must be 16-byte aligned");
    const int nch = col / 8;
    AVR_REQUIRE(N >= 0 && N * nch < (int64_t(1) << 31), "avr_concat_fwd: too many rows");
    if (N == 0) return 0;
    const uint64_t threads = (uint64_t)N * nch;
    hipLaunchKernelGGL(concat_fwd_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       as_stream(stream), (uint32_t)N, nch, t, out, out_dtype);
    return check_launch("avr_concat_fwd");
}

extern "C" int avr_concat_bwd(int64_t N, int32_t n_src, const avr_concat_src* src, const void* grad_out,
                              int32_t grad_dtype, float* workspace, void* stream) {
    AVR_REQUIRE(src && grad_out && n_src >= 1 && n_src <= kMaxSrc && dtype_ok(grad_dtype),
                "avr_concat_bwd: bad arguments");
    int ldo = 0;
    for (int i = 0; i < n_src; ++i) ldo += src[i].width;
    AVR_REQUIRE(N >= 0 && N * ldo < (int64_t(1) << 31), "avr_concat_bwd: too many rows");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(grad_out) % 16 == 0, "avr_concat_bwd: grad_out must be 16-byte aligned");
    hipStream_t st = as_stream(stream);
    int col = 0;
    for (int i = 0; i < n_src; ++i) {
        const avr_concat_src& s = src[i];
        AVR_REQUIRE(dtype_ok(s.dtype) && s.rows_div >= 1 && s.width % 8 == 0 && N % s.rows_div == 0,
                    "avr_concat_bwd: bad source (rows_div must divide N)");
        if (s.grad) {
            AVR_REQUIRE(reinterpret_cast<uintptr_t>(s.grad) % 16 == 0, "avr_concat_bwd: grad not aligned");
            const uint32_t n_out = (uint32_t)(N / s.rows_div);
            const int w8 = s.width / 8;
            if (s.rows_div > 1 && s.split > 1 && s.rows_div % s.split == 0) {
                // two passes: groups of rows_div/split rows into the fp32
                // workspace, then groups of split partial rows
                AVR_REQUIRE(workspace != nullptr, "avr_concat_bwd: split needs a workspace");
                const int d1 = s.rows_div / s.split;
                if (int e = launch_group_sum((uint32_t)(N / d1), d1, w8, grad_out, grad_dtype, ldo, col,
                                             workspace, AVR_DTYPE_F32, st))
                    return e;
                if (int e = launch_group_sum(n_out, s.split, w8, workspace, AVR_DTYPE_F32, s.width, 0, s.grad,
                                             s.dtype, st))
                    return e;
            } else if (int e = launch_group_sum(n_out, s.rows_div, w8, grad_out, grad_dtype, ldo, col, s.grad,
                                                s.dtype, st)) {
                return e;
            }
        }
        col += s.width;
    }
    return 0;
}
