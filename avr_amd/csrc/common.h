// Shared device helpers for the AVR HIP library (gfx950).
//
// This translation unit family is compiled with -ffp-contract=off: every
// a*b+c below is two roundings unless written as fmaf(), because the
// reference's torch-CPU ops round each op separately
// and the integer delays are sensitive to single-ulp differences.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <type_traits>
#include <stdint.h>
#include <string>

#include "avr_hip.h"

namespace avr {

// ---------------------------------------------------------------- errors
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);
// compute units of the current device, queried once per device
// (std::call_once: safe from concurrent host threads, e.g. nn.DataParallel)
int device_cus();

#define AVR_REQUIRE(cond, msg)                          \
    do {                                                \
        if (!(cond)) return ::avr::fail(AVR_E_ARG, msg); \
    } while (0)

// irfft of B spectra [B][F][2] -> [B][2(F-1)], and of a second batch
// (spec2 -> ir2, may be null) in the same launch (render_fwd.hip).
int launch_irfft(int B, int F, const float* spec, const float* spec2, const float* tw, float* ir,
                 float* ir2, void* stream);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- MFMA operand hold
// A register an MFMA reads as SrcB must not be rewritten while that MFMA may
// still wait in the matrix pipe's queue (the bf16x3
// DFT returned stale B-operand lanes when the compiler refilled a B register
// right behind a queued MFMA).  At the end of an MFMA chain: every MFMA of
// the chain issues first (sched_barrier: nothing crosses), then 8 wait states
// (one 32x32 MFMA's passes), then each operand is used once more, so its
// register is not reallocated before that point.  tests/test_isa_audit.py
// checks the compiled library for the pattern.
__device__ __forceinline__ void mfma_queue_wait() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7");
}
template <typename T>
__device__ __forceinline__ void keep_live(const T& v) {
    asm volatile("" ::"v"(v));
}

// ---------------------------------------------------------------- dtypes
__device__ __forceinline__ float load_f(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float load_f(const __half* p, int64_t i) { return __half2float(p[i]); }
__device__ __forceinline__ float load_f(const __hip_bfloat16* p, int64_t i) {
    return __bfloat162float(p[i]);
}
__device__ __forceinline__ void store_f(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void store_f(__half* p, int64_t i, float v) { p[i] = __float2half(v); }
__device__ __forceinline__ void store_f(__hip_bfloat16* p, int64_t i, float v) {
    p[i] = __float2bfloat16(v);  // round to nearest even
}
// bf16 pair packed in a dword -> two floats (exact)
__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
// fp16 pair packed in a dword -> two floats (exact)
__device__ __forceinline__ float f16_lo(uint32_t u) { return __half2float(__ushort_as_half((unsigned short)(u & 0xffffu))); }
__device__ __forceinline__ float f16_hi(uint32_t u) { return __half2float(__ushort_as_half((unsigned short)(u >> 16))); }

// element k of a dword-packed row of 16-bit values of type T (fp16 or bf16)
template <typename T>
__device__ __forceinline__ float unpack16(uint32_t u, int hi) {
    if constexpr (std::is_same<T, __half>::value)
        return hi ? f16_hi(u) : f16_lo(u);
    else
        return hi ? bf16_hi(u) : bf16_lo(u);
}
// two floats -> a dword of two 16-bit values of type T (round to nearest even)
template <typename T>
__device__ __forceinline__ uint32_t pack16(float a, float b) {
    if constexpr (std::is_same<T, __half>::value) {
        return (uint32_t)__half_as_ushort(__float2half(a)) | ((uint32_t)__half_as_ushort(__float2half(b)) << 16);
    } else {
        const __hip_bfloat16 x = __float2bfloat16(a), y = __float2bfloat16(b);
        return (uint32_t)(*reinterpret_cast<const uint16_t*>(&x)) |
               ((uint32_t)(*reinterpret_cast<const uint16_t*>(&y)) << 16);
    }
}

// 16-byte vectors of signal elements as floats: 4 x fp32 or 8 x fp16/bf16.
// load() is non-temporal (the signal is streamed once per pass and should
// not evict the tables and partials from L2/MALL); store16() is a plain
// 16-byte store, store16_nt() a streaming one.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
    static constexpr int N = 4;
    using raw = f32x4;
    __device__ static void cvt(const raw& v, float* o) {
        o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
    }
    __device__ static raw pack(const float* o) { return raw{o[0], o[1], o[2], o[3]}; }
};
template <>
struct Vec16<__half> {
    static constexpr int N = 8;
    using raw = u32x4;
    __device__ static void cvt(const raw& v, float* o) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t u = v[i];
            const float2 f = __half22float2(*reinterpret_cast<const __half2*>(&u));
            o[2 * i] = f.x;
            o[2 * i + 1] = f.y;
        }
    }
    __device__ static raw pack(const float* o) {
        raw v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const __half2 h = __floats2half2_rn(o[2 * i], o[2 * i + 1]);
            v[i] = *reinterpret_cast<const uint32_t*>(&h);
        }
        return v;
    }
};
template <>
struct Vec16<__hip_bfloat16> {
    static constexpr int N = 8;
    using raw = u32x4;
    __device__ static void cvt(const raw& v, float* o) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i] = bf16_lo(v[i]);
            o[2 * i + 1] = bf16_hi(v[i]);
        }
    }
    __device__ static raw pack(const float* o) {
        raw v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const __hip_bfloat16 a = __float2bfloat16(o[2 * i]);
            const __hip_bfloat16 b = __float2bfloat16(o[2 * i + 1]);
            v[i] = (uint32_t)(*reinterpret_cast<const uint16_t*>(&a)) |
                   ((uint32_t)(*reinterpret_cast<const uint16_t*>(&b)) << 16);
        }
        return v;
    }
};
template <typename T>
__device__ __forceinline__ void load16_nt(const T* p, float* o) {
    using V = Vec16<T>;
    V::cvt(__builtin_nontemporal_load(reinterpret_cast<const typename V::raw*>(p)), o);
}
// Streaming 16-byte load through a buffer resource whose base is the current
// (wave-uniform) row: a lane whose byte offset is >= nbytes gets zeros and
// issues no memory traffic.  That masks chunks without control flow, so all
// loads of an unrolled batch stay in flight together.
constexpr uint32_t kSkip = 0x80000000u;  // byte offset of a masked lane
template <typename T>
__device__ __forceinline__ void load16_masked(const T* row, uint32_t nbytes, uint32_t off,
                                              float* o) {
    using V = Vec16<T>;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)row, (short)0, (int)nbytes, 0x00020000);
    // aux = 2: non-temporal (gfx94x/gfx950 "nt")
    V::cvt(__builtin_bit_cast(typename V::raw,
                              __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)off, 0, 2)),
           o);
}
template <typename T>
__device__ __forceinline__ void store16(T* p, const float* o) {
    using V = Vec16<T>;
    *reinterpret_cast<typename V::raw*>(p) = V::pack(o);
}
template <typename T>
__device__ __forceinline__ void store16_nt(T* p, const float* o) {
    using V = Vec16<T>;
    __builtin_nontemporal_store(V::pack(o), reinterpret_cast<typename V::raw*>(p));
}

// ---------------------------------------------------------------- geometry
// torch.linspace(a, b, n)[i] on CPU: step = (b-a)/(n-1) in fp32, lower half
// a + step*i, upper half b - step*(n-1-i), each a single fused rounding.
__device__ __forceinline__ float linspace_at(float a, float b, int n, int i) {
    if (n == 1) return a;
    const float step = (b - a) / (float)(n - 1);
    return (i < n / 2) ? fmaf(step, (float)i, a) : fmaf(-step, (float)(n - 1 - i), b);
}

// normalize_points (renderer.py:127-128): 2*(x-lo)/span - 1, op by op.
__device__ __forceinline__ float to_unit(float x, float lo, float span) {
    float y = x - lo;
    y = 2.0f * y;
    y = y / span;
    return y - 1.0f;
}

// denormalize_points (renderer.py:130-131): (q+1)/2*span + lo, op by op.
__device__ __forceinline__ float from_unit(float q, float lo, float span) {
    float y = q + 1.0f;
    y = y / 2.0f;
    y = y * span;
    return y + lo;
}

// Integer source delay of one ray-sample (renderer.py:55-58, 86-87):
// world point o + dir*d, normalized; tx normalized; denormalized gap; norm
// as torch's vector_norm reduces it (fma chain); *fs/speed; round-half-even;
// clamp to [0, T-1].
__device__ __forceinline__ int source_delay(const avr_render_params& p, const float o[3],
                                            const float txn[3], const float dir[3], float d) {
    float g[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float world = o[c] + dir[c] * d;
        const float pn = to_unit(world, p.lo, p.span);
        g[c] = from_unit(txn[c] - pn, p.lo, p.span);
    }
    const float n2 = fmaf(g[2], g[2], fmaf(g[1], g[1], g[0] * g[0]));
    const float idx = (sqrtf(n2) * p.fs) / p.speed;
    float r = rintf(idx);
    r = fminf(fmaxf(r, 0.0f), (float)(p.T - 1));
    return (int)r;
}

// rays of the render core (a shard of the sphere when rays are split over GPUs)
__host__ __device__ inline int n_rays(const avr_render_params& p) { return p.n_rays; }

// Copy n float2 from global into LDS with every load of a round in flight
// before the first LDS store (a plain strided loop serialises load->store
// pairs).  Indices are clamped so no load sits behind a branch.
template <int THREADS>
__device__ __forceinline__ void stage_table(float2* __restrict__ dst, const float2* __restrict__ src,
                                            int n) {
    constexpr int R = 8;
    for (int base = 0; base < n; base += R * THREADS) {
        float2 v[R];
#pragma unroll
        for (int i = 0; i < R; ++i) v[i] = src[min(base + i * THREADS + (int)threadIdx.x, n - 1)];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int j = base + i * THREADS + (int)threadIdx.x;
            if (j < n) dst[j] = v[i];
        }
    }
}
// receiver-side depth and integer delay of sample s (renderer.py:64-70):
// d = linspace(0,1,S)[s]*(far-near)+near, shift = round(fs*d/speed).
// Every kernel recomputes it with the same op sequence as tables_kernel.
__device__ __forceinline__ float depth_at(const avr_render_params& p, int s) {
    return linspace_at(0.0f, 1.0f, p.n_samples, s) * p.depth_scale + p.depth_offset;
}
__device__ __forceinline__ int receiver_shift(const avr_render_params& p, int s) {
    return (int)rintf((p.fs * depth_at(p, s)) / p.speed);
}
// last+1 sample time kept by the tail mask (renderer.py:72): t < T-1-shift
__device__ __forceinline__ int tail_limit(const avr_render_params& p, int s) {
    return p.T - 1 - receiver_shift(p, s);
}
// all rays of the sphere (ray generation)
__host__ __device__ inline int grid_rays(const avr_render_params& p) { return p.n_azi * p.n_ele + 2; }

}  // namespace avr
