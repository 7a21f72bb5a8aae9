// Multiresolution hash-grid encoding (a5) for gfx950.
//
// Replaces tcnn.Encoding(3, {"otype": "HashGrid", ...}) used by the
// reference's networks (model.py:66-68, 191, 219-220, 258-263, 315-324).
// tinycudann is not vendored in the reference; the semantics follow upstream
// tiny-cuda-nn's GridEncoding (Hash grid, N-linear interpolation, coherent
// prime hash, +0.5 staggering, per-level size min(res^3 rounded to 8,
// 2^log2_hashmap_size)) — parity UNPINNED (no reference fixture exists),
// checked against the repo's own restatement oracle/hashgrid_oracle.py.
//
// One thread per (point, level) with the level index fastest, so a wavefront
// covers 64/L points x all levels: the 8-byte feature pairs are written
// fully coalesced, the coordinates are shared through L1, and the gathers of
// one point's levels go to L2/MALL-resident tables (<= 2 MiB fp32 per level).
// Weights and coordinates are fp32; the corner sum runs in the table type
// (fp16 tables: half FMAs, as tcnn's fp16 GridEncoding; CornerAcc).
#include "common.h"

using namespace avr;

namespace {

constexpr int kMaxLevels = 32;

struct LevelTable {
    int64_t offset[kMaxLevels + 1];
    float scale[kMaxLevels];
    uint32_t res[kMaxLevels];
};

__device__ __forceinline__ uint32_t grid_index(uint32_t size, uint32_t res, uint32_t x, uint32_t y,
                                               uint32_t z) {
    // dense index while it fits the level, coherent-prime hash otherwise
    uint64_t stride = 1;
    uint32_t index = 0;
    const uint32_t c[3] = {x, y, z};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        if (stride > size) break;
        index += c[d] * (uint32_t)stride;
        stride *= res;
    }
    if (size < stride) index = (x * 1u) ^ (y * 2654435761u) ^ (z * 805459861u);
    return index % size;
}

template <typename Tp>
__device__ __forceinline__ float2 load_pair(const Tp* params, int64_t entry);
template <>
__device__ __forceinline__ float2 load_pair<float>(const float* params, int64_t entry) {
    return *reinterpret_cast<const float2*>(params + 2 * entry);
}
template <>
__device__ __forceinline__ float2 load_pair<__half>(const __half* params, int64_t entry) {
    return __half22float2(*reinterpret_cast<const __half2*>(params + 2 * entry));
}

// Corner accumulation in the table type, as tcnn's kernel_grid does
// (`result = fma((T)weight, grid_val(local_pos), result)`, corners in index
// order with the x bit fastest): fp32 tables accumulate with fp32 fmaf; fp16
// tables round the trilinear weight to half and accumulate with a packed half
// FMA (v_pk_fma_f16: one rounding per feature per corner), so an fp16
// encoding holds exactly the half values tcnn's fp16 GridEncoding returns.
template <typename Tp>
struct CornerAcc;
template <>
struct CornerAcc<float> {
    using raw = float2;
    float2 a = make_float2(0.0f, 0.0f);
    __device__ __forceinline__ static raw load(const float* table, uint32_t e) {
        return *reinterpret_cast<const float2*>(table + 2 * (size_t)e);
    }
    __device__ __forceinline__ void add(float w, raw v) {
        a.x = fmaf(w, v.x, a.x);
        a.y = fmaf(w, v.y, a.y);
    }
    __device__ __forceinline__ float2 get() const { return a; }
};
template <>
struct CornerAcc<__half> {
    using raw = __half2;
    __half2 a = __float2half2_rn(0.0f);
    __device__ __forceinline__ static raw load(const __half* table, uint32_t e) {
        return *reinterpret_cast<const __half2*>(table + 2 * (size_t)e);
    }
    __device__ __forceinline__ void add(float w, raw v) {
        // v_pk_fma_f16 explicitly: left to itself the compiler folds the
        // weight's float->half conversion into v_fma_mixlo_f16, which rounds
        // the fma to f32 and then to f16 (double rounding: ~1 element in 10^4
        // one half-ulp off tcnn's single-rounded __hfma2)
        const __half2 w2 = __float2half2_rn(w);
        uint32_t r, wu, vu, au;
        __builtin_memcpy(&wu, &w2, 4);
        __builtin_memcpy(&vu, &v, 4);
        __builtin_memcpy(&au, &a, 4);
        asm("v_pk_fma_f16 %0, %1, %2, %3" : "=v"(r) : "v"(wu), "v"(vu), "v"(au));
        __builtin_memcpy(&a, &r, 4);
    }
    __device__ __forceinline__ float2 get() const { return __half22float2(a); }  // exact
};

template <typename To>
__device__ __forceinline__ void store_pair(To* out, int64_t i, float2 v);
template <>
__device__ __forceinline__ void store_pair<float>(float* out, int64_t i, float2 v) {
    *reinterpret_cast<float2*>(out + 2 * i) = v;
}
template <>
__device__ __forceinline__ void store_pair<__half>(__half* out, int64_t i, float2 v) {
    *reinterpret_cast<__half2*>(out + 2 * i) = __floats2half2_rn(v.x, v.y);
}

// avr_hashgrid_fwd switches to the level-major dispatch from this many points
// (AVR_HASHGRID_LM_MIN overrides; experiments)
constexpr int64_t kLevelMajorMinPointsDefault = 16384;
inline int64_t lm_min_points() {
    static const int64_t v = [] {
        const char* e = getenv("AVR_HASHGRID_LM_MIN");
        return e ? (int64_t)atoll(e) : kLevelMajorMinPointsDefault;
    }();
    return v;
}

// grouped corner loads in the level-major forward (AVR_HASHGRID_GROUP=0
// turns them off; experiments)
inline bool group_loads() {
    static const bool v = [] {
        const char* e = getenv("AVR_HASHGRID_GROUP");
        return !(e && e[0] == '0');
    }();
    return v;
}

struct Corner {
    float pos[3];
    uint32_t grid[3];
};

__device__ __forceinline__ Corner locate(const float* x, float scale) {
    Corner c;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float p = fmaf(scale, x[d], 0.5f);
        const float fl = floorf(p);
        c.grid[d] = (uint32_t)(int)fl;
        c.pos[d] = p - fl;
    }
    return c;
}

template <typename Tp, typename To>
__global__ __launch_bounds__(256) void hashgrid_fwd_kernel(int64_t N, int L,
                                                           const float* __restrict__ x,
                                                           const Tp* __restrict__ params,
                                                           LevelTable lt, To* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= N * L) return;
    const int64_t i = q / L;
    const int l = (int)(q % L);
    const float xi[3] = {x[i * 3 + 0], x[i * 3 + 1], x[i * 3 + 2]};
    const Corner c = locate(xi, lt.scale[l]);
    const uint32_t size = (uint32_t)(lt.offset[l + 1] - lt.offset[l]);
    const uint32_t res = lt.res[l];
    const Tp* table = params + 2 * lt.offset[l];
    CornerAcc<Tp> acc;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float wgt = 1.0f;
        uint32_t g[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (k & (1 << d)) {
                wgt *= c.pos[d];
                g[d] = c.grid[d] + 1;
            } else {
                wgt *= 1.0f - c.pos[d];
                g[d] = c.grid[d];
            }
        }
        acc.add(wgt, CornerAcc<Tp>::load(table, grid_index(size, res, g[0], g[1], g[2])));
    }
    store_pair(out, q, acc.get());
}

// Level-major forward for inference: grid (points / 256, L), blockIdx.y =
// level, so the blocks in flight work on one or two levels at a time and the
// level's table (<= 2 MiB fp32) stays resident in each XCD's 4 MiB L2
// instead of all L tables (36 MiB for the MeshRIR position grid) streaming
// from the Infinity Cache.  out is level-major [L][N][2] (coalesced stores);
// consumers read feature pair l of point i at out[l*N + i].
//
// ROW_MAJOR: the same level-major dispatch writing the row-major [N][L][2]
// output of hashgrid_fwd_kernel (avr_hashgrid_fwd for large N: training's
// per-sample grids).  The 8-byte stores are strided, but they are 1/8 of the
// gathered bytes; the gathers are what the L2-resident level saves.
//
// GROUP (fp16 tables): the two x-neighbour corners of a cell edge usually
// sit in one aligned 16-byte group of 4 table entries: on hashed levels x
// enters the hash with prime 1, so x -> x+1 flips only the trailing bits of
// the entry (x mod 4 != 3: same group); on dense levels the entry is the
// next one.  Each edge therefore issues one 16-byte load of the group
// holding its first corner, and a second (exec-masked) load only in the
// lanes whose second corner lies outside it: fewer address lookups per wave
// than 8 separate loads, the same values, the same fmaf order (bit-identical
// output).  Needs a 16-byte aligned table base (level sizes are multiples of
// 8 entries); the host checks.
template <typename Tp>
struct EntryGroup;
template <>
struct EntryGroup<__half> {
    static constexpr uint32_t kN = 4;
    uint32_t d[4];
    __device__ __forceinline__ void load(const __half* table, uint32_t e) {
        const uint4 v = *reinterpret_cast<const uint4*>(table + 2 * (e & ~(kN - 1)));
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
    __device__ __forceinline__ __half2 get(uint32_t e) const {
        const uint32_t j = e & (kN - 1);
        const uint32_t v = j == 0 ? d[0] : j == 1 ? d[1] : j == 2 ? d[2] : d[3];
        __half2 h;
        __builtin_memcpy(&h, &v, 4);
        return h;
    }
};

template <typename Tp, typename To, bool ROW_MAJOR = false, bool GROUP = false>
__global__ __launch_bounds__(256) void hashgrid_fwd_lm_kernel(int64_t N, const float* __restrict__ x,
                                                              const Tp* __restrict__ params,
                                                              LevelTable lt, To* __restrict__ out) {
    const int l = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const float xi[3] = {x[i * 3 + 0], x[i * 3 + 1], x[i * 3 + 2]};
    const Corner c = locate(xi, lt.scale[l]);
    const uint32_t size = (uint32_t)(lt.offset[l + 1] - lt.offset[l]);
    const uint32_t res = lt.res[l];
    const Tp* table = params + 2 * lt.offset[l];
    CornerAcc<Tp> acc;
    // corner weights and entries in the order k = 0..7 (x bit fastest)
    float wgt[8];
    uint32_t ent[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float w = 1.0f;
        uint32_t g[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (k & (1 << d)) {
                w *= c.pos[d];
                g[d] = c.grid[d] + 1;
            } else {
                w *= 1.0f - c.pos[d];
                g[d] = c.grid[d];
            }
        }
        wgt[k] = w;
        ent[k] = grid_index(size, res, g[0], g[1], g[2]);
    }
    if constexpr (GROUP) {
        constexpr uint32_t kN = EntryGroup<Tp>::kN;
        EntryGroup<Tp> grp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) grp[j].load(table, ent[2 * j]);
        using raw = typename CornerAcc<Tp>::raw;
        raw far[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            far[j] = grp[j].get(ent[2 * j]);
            if ((ent[2 * j + 1] ^ ent[2 * j]) >= kN) far[j] = CornerAcc<Tp>::load(table, ent[2 * j + 1]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const raw v0 = grp[j].get(ent[2 * j]);
            const raw v1 = ((ent[2 * j + 1] ^ ent[2 * j]) >= kN) ? far[j] : grp[j].get(ent[2 * j + 1]);
            acc.add(wgt[2 * j], v0);
            acc.add(wgt[2 * j + 1], v1);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc.add(wgt[k], CornerAcc<Tp>::load(table, ent[k]));
    }
    store_pair(out, ROW_MAJOR ? i * (int64_t)gridDim.y + l : (int64_t)l * N + i, acc.get());
}

// Backward: scatter-add of w_corner * dL/dy into the tables.
//
// Float atomics execute at the memory side and cost one request per 64-B
// segment a wave-instruction touches (MI355X_MICROARCH.md, Global float
// atomics: 64 lanes in 64 different rows are ~17x slower than 64 contiguous
// dwords).  So a lane owns ONE dword: (point, corner k, feature f), 16 lanes
// per point, lane order (k, f) with the x-corner bit next to the feature
// bit.  The 4 dwords of an x-neighbour pair are adjacent in the table (dense
// levels: consecutive entries; hashed levels: x enters the hash with prime 1,
// so x and x+1 usually differ only in the low bits of the entry), so one
// wave-instruction (4 points x 16 dwords) touches ~4 segments per point
// instead of 16 requests per point for a lane-per-point layout.
//
// Points of a wave that hit the same dword (consecutive samples of a ray in
// one coarse cell) are first summed over runs of equal addresses across the
// 4 points (head flags at lane stride 16) and only the last one adds.
template <typename Tg>
__global__ __launch_bounds__(256) void hashgrid_bwd_kernel(int64_t N, int L,
                                                           const float* __restrict__ x,
                                                           const Tg* __restrict__ gout,
                                                           LevelTable lt,
                                                           float* __restrict__ gparams) {
    const int l = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int slot = threadIdx.x & 15;
    const int k = slot >> 1, f = slot & 1;
    const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
    const bool live = i < N;
    const int64_t ic = live ? i : N - 1;
    const float xi[3] = {x[ic * 3 + 0], x[ic * 3 + 1], x[ic * 3 + 2]};
    const float g = live ? load_f(gout, ic * (2 * L) + 2 * l + f) : 0.0f;
    const Corner c = locate(xi, lt.scale[l]);
    const uint32_t size = (uint32_t)(lt.offset[l + 1] - lt.offset[l]);
    const uint32_t res = lt.res[l];
    float wgt = 1.0f;
    uint32_t gg[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        if (k & (1 << d)) {
            wgt *= c.pos[d];
            gg[d] = c.grid[d] + 1;
        } else {
            wgt *= 1.0f - c.pos[d];
            gg[d] = c.grid[d];
        }
    }
    const uint32_t e = 2u * grid_index(size, res, gg[0], gg[1], gg[2]) + (uint32_t)f;
    float v = wgt * g;
    // runs of equal e over the wave's 4 points (same slot: lanes 16 apart)
    const int p = lane >> 4;
    const uint32_t prev = __shfl_up(e, 16, 64);
    const bool head = p == 0 || prev != e;
    const unsigned long long heads = __ballot(head);
    int start = p;
    while (!((heads >> (16 * start + slot)) & 1ull)) --start;  // <= 3 steps
#pragma unroll
    for (int off = 16; off < 64; off <<= 1) {
        const float o = __shfl_up(v, off, 64);
        if (lane - off >= 16 * start + slot) v += o;
    }
    const bool tail = p == 3 || ((heads >> (lane + 16)) & 1ull);
    if (tail && v != 0.0f) atomicAdd(gparams + 2 * lt.offset[l] + e, v);
}

int make_table(int L, const int64_t* off, const float* scale, const int32_t* res, LevelTable* lt) {
    if (L < 1 || L > kMaxLevels) return fail(AVR_E_ARG, "hashgrid: n_levels out of range (1..32)");
    for (int l = 0; l <= L; ++l) lt->offset[l] = off[l];
    for (int l = 0; l < L; ++l) {
        lt->scale[l] = scale[l];
        lt->res[l] = (uint32_t)res[l];
        if (off[l + 1] <= off[l]) return fail(AVR_E_ARG, "hashgrid: empty level");
    }
    return 0;
}

template <typename Tp, typename To, bool ROW_MAJOR>
void launch_lm(dim3 grid, hipStream_t st, int64_t N, const float* x, const void* params, LevelTable lt,
               void* out, bool grp) {
    if constexpr (std::is_same_v<Tp, __half>) {
        if (grp) {
            hipLaunchKernelGGL((hashgrid_fwd_lm_kernel<Tp, To, ROW_MAJOR, true>), grid, dim3(256), 0, st, N,
                               x, (const Tp*)params, lt, (To*)out);
            return;
        }
    }
    hipLaunchKernelGGL((hashgrid_fwd_lm_kernel<Tp, To, ROW_MAJOR, false>), grid, dim3(256), 0, st, N, x,
                           (const Tp*)params, lt, (To*)out);
}

// Level-major forward launch; grouped corner loads for fp16 tables whose
// base is 16-byte aligned (level offsets are multiples of 8 entries).  fp32
// tables keep the 8-byte loads: a 16-byte group holds only 2 entries there
// and measured slower (config-2 points: 102 -> 119 us level-major, 141 ->
// 156 us row-major); fp16: 113-117 -> 103-106 us level-major, 138-140 ->
// 116-118 us row-major (profiles/r02_hashgrid_group_ab.jsonl)
template <bool ROW_MAJOR>
int launch_fwd_lm(dim3 grid, hipStream_t st, int64_t N, const float* x, const void* params,
                  int32_t param_dtype, const LevelTable& lt, void* out, int32_t out_dtype) {
    const bool grp = group_loads() && ((uintptr_t)params & 15) == 0;
    if (param_dtype == AVR_DTYPE_F32 && out_dtype == AVR_DTYPE_F32)
        launch_lm<float, float, ROW_MAJOR>(grid, st, N, x, params, lt, out, grp);
    else if (param_dtype == AVR_DTYPE_F32 && out_dtype == AVR_DTYPE_F16)
        launch_lm<float, __half, ROW_MAJOR>(grid, st, N, x, params, lt, out, grp);
    else if (param_dtype == AVR_DTYPE_F16 && out_dtype == AVR_DTYPE_F16)
        launch_lm<__half, __half, ROW_MAJOR>(grid, st, N, x, params, lt, out, grp);
    else if (param_dtype == AVR_DTYPE_F16 && out_dtype == AVR_DTYPE_F32)
        launch_lm<__half, float, ROW_MAJOR>(grid, st, N, x, params, lt, out, grp);
    else
        return fail(AVR_E_ARG, "avr_hashgrid_fwd: unknown dtype");
    return 0;
}

}  // namespace

// level_offset / level_scale / level_res are HOST pointers (small metadata,
// passed by value into the kernel argument block).
extern "C" int avr_hashgrid_fwd(int64_t N, int32_t n_levels, const float* x, const void* params,
                                int32_t param_dtype, const int64_t* level_offset,
                                const float* level_scale, const int32_t* level_res, void* out,
                                int32_t out_dtype, void* stream) {
    AVR_REQUIRE(N >= 0 && x && params && level_offset && level_scale && level_res && out,
                "avr_hashgrid_fwd: bad args");
    if (N == 0) return 0;
    LevelTable lt;
    if (int e = make_table(n_levels, level_offset, level_scale, level_res, &lt)) return e;
    const int64_t work = N * n_levels;
    const dim3 grid((unsigned)((work + 255) / 256));
    hipStream_t st = as_stream(stream);
    const int L = n_levels;
    // many points: level-major dispatch (one level's table L2-resident at a
    // time), same values and output layout (tools/probe_hashgrid.py)
    if (N >= lm_min_points()) {
        const dim3 glm((unsigned)((N + 255) / 256), (unsigned)L);
        if (int e = launch_fwd_lm<true>(glm, st, N, x, params, param_dtype, lt, out, out_dtype)) return e;
        return check_launch("avr_hashgrid_fwd");
    }
    if (param_dtype == AVR_DTYPE_F32 && out_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL((hashgrid_fwd_kernel<float, float>), grid, dim3(256), 0, st, N, L, x,
                           (const float*)params, lt, (float*)out);
    else if (param_dtype == AVR_DTYPE_F32 && out_dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL((hashgrid_fwd_kernel<float, __half>), grid, dim3(256), 0, st, N, L, x,
                           (const float*)params, lt, (__half*)out);
    else if (param_dtype == AVR_DTYPE_F16 && out_dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL((hashgrid_fwd_kernel<__half, __half>), grid, dim3(256), 0, st, N, L, x,
                           (const __half*)params, lt, (__half*)out);
    else if (param_dtype == AVR_DTYPE_F16 && out_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL((hashgrid_fwd_kernel<__half, float>), grid, dim3(256), 0, st, N, L, x,
                           (const __half*)params, lt, (float*)out);
    else
        return fail(AVR_E_ARG, "avr_hashgrid_fwd: unknown dtype");
    return check_launch("avr_hashgrid_fwd");
}

extern "C" int avr_hashgrid_bwd(int64_t N, int32_t n_levels, const float* x, const void* grad_out,
                                int32_t grad_dtype, const int64_t* level_offset,
                                const float* level_scale, const int32_t* level_res,
                                float* grad_params, void* stream) {
    AVR_REQUIRE(N >= 0 && x && grad_out && level_offset && level_scale && level_res && grad_params,
                "avr_hashgrid_bwd: bad args");
    if (N == 0) return 0;
    LevelTable lt;
    if (int e = make_table(n_levels, level_offset, level_scale, level_res, &lt)) return e;
    const dim3 grid((unsigned)((N + 15) / 16), (unsigned)n_levels);  // 16 lanes per point
    hipStream_t st = as_stream(stream);
    if (grad_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL(hashgrid_bwd_kernel<float>, grid, dim3(256), 0, st, N, (int)n_levels, x,
                           (const float*)grad_out, lt, grad_params);
    else if (grad_dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL(hashgrid_bwd_kernel<__half>, grid, dim3(256), 0, st, N, (int)n_levels,
                           x, (const __half*)grad_out, lt, grad_params);
    else
        return fail(AVR_E_ARG, "avr_hashgrid_bwd: unknown grad dtype");
    return check_launch("avr_hashgrid_bwd");
}

extern "C" int avr_hashgrid_fwd_lm(int64_t N, int32_t n_levels, const float* x, const void* params,
                                   int32_t param_dtype, const int64_t* level_offset,
                                   const float* level_scale, const int32_t* level_res, void* out,
                                   int32_t out_dtype, void* stream) {
    AVR_REQUIRE(N >= 0 && x && params && level_offset && level_scale && level_res && out,
                "avr_hashgrid_fwd_lm: bad args");
    if (N == 0) return 0;
    LevelTable lt;
    if (int e = make_table(n_levels, level_offset, level_scale, level_res, &lt)) return e;
    const dim3 grid((unsigned)((N + 255) / 256), (unsigned)n_levels);
    hipStream_t st = as_stream(stream);
    if (int e = launch_fwd_lm<false>(grid, st, N, x, params, param_dtype, lt, out, out_dtype)) return e;
    return check_launch("avr_hashgrid_fwd_lm");
}

// ----------------------------------------------------------------------------
// Per-ray / per-pose first-layer bias of AVRModel's signal network at
// inference (avr_amd/model.py _trunk_fused_h1): for every ray of every pose
//
//   e_dir = bf16(enc_dtype(dir_grid((view[b, r*S] + 1) / 2)))     [2*Ld]
//   e_tx  = bf16(enc_dtype(tx_grid((tx[b, 0] + 1) / 2)))           [2*Lt]
//   bias[b*R + r][o] = sum_k e_dir[k] w_dir[k][o] + sum_k e_tx[k] w_tx[k][o]
//
// (the view direction repeats over a ray's samples and tx over a pose's,
// model.py:221 concatenates both to every sample).  One launch instead of
// the ~12 small torch kernels of the same arithmetic: the row selection, the
// [0, 1] map, two small grids, the fp16 -> bf16 -> fp32 casts, two skinny
// GEMMs and their sum.  Each workgroup does kBiasRays rays: encodings into
// LDS, then each thread walks k for its outputs with the rays' sums in
// registers (k ascending: a fixed order), the weight rows of 8 k in flight
// at a time (a k-step waits on an L2 load otherwise: with 16 rays per
// workgroup and the loads one by one this kernel took 49 us for 1024 rays).
namespace {

constexpr int kBiasRays = 4;  // 256 workgroups for config 2's 1024 rays

template <typename Tp>
__device__ __forceinline__ float2 encode_point_level(const float* xi, const Tp* params, const LevelTable& lt, int l) {
    const Corner c = locate(xi, lt.scale[l]);
    const uint32_t size = (uint32_t)(lt.offset[l + 1] - lt.offset[l]);
    const uint32_t res = lt.res[l];
    const Tp* table = params + 2 * lt.offset[l];
    CornerAcc<Tp> acc;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float wgt = 1.0f;
        uint32_t g[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (k & (1 << d)) {
                wgt *= c.pos[d];
                g[d] = c.grid[d] + 1;
            } else {
                wgt *= 1.0f - c.pos[d];
                g[d] = c.grid[d];
            }
        }
        acc.add(wgt, CornerAcc<Tp>::load(table, grid_index(size, res, g[0], g[1], g[2])));
    }
    return acc.get();
}

__device__ __forceinline__ float round_feature(float v, bool f16, bool mlp_f16) {
    if (f16) v = __half2float(__float2half(v));               // the encoding's output dtype
    return mlp_f16 ? __half2float(__float2half(v))            // the MLP's 16-bit input
                   : __bfloat162float(__float2bfloat16(v));
}

template <typename Tp>
__global__ __launch_bounds__(256) void ray_pose_bias_kernel(int B, int R, int S, const float* __restrict__ view,
                                                            const float* __restrict__ tx, const Tp* __restrict__ dp,
                                                            LevelTable dl, int dL, const Tp* __restrict__ tp,
                                                            LevelTable tl, int tL, int f16, int mlp_f16,
                                                            const float* __restrict__ wd,
                                                            const float* __restrict__ wt, int nout,
                                                            float* __restrict__ bias) {
    __shared__ float e[kBiasRays][2][2 * kMaxLevels];
    const int64_t g0 = (int64_t)blockIdx.x * kBiasRays;
    const int nr = (int)min((int64_t)kBiasRays, (int64_t)B * R - g0);
    for (int q = threadIdx.x; q < kBiasRays * 2 * kMaxLevels; q += 256) {
        const int j = q / (2 * kMaxLevels), rem = q % (2 * kMaxLevels);
        const int which = rem / kMaxLevels, l = rem % kMaxLevels;
        if (j >= nr || l >= (which ? tL : dL)) continue;
        const int64_t gr = g0 + j;
        const int64_t b = gr / R, r = gr % R;
        const float* src = which ? tx + b * R * S * 3 : view + (b * R * S + r * S) * 3;
        const float xi[3] = {(src[0] + 1.0f) / 2.0f, (src[1] + 1.0f) / 2.0f, (src[2] + 1.0f) / 2.0f};
        const float2 v = which ? encode_point_level(xi, tp, tl, l) : encode_point_level(xi, dp, dl, l);
        e[j][which][2 * l] = round_feature(v.x, f16, mlp_f16);
        e[j][which][2 * l + 1] = round_feature(v.y, f16, mlp_f16);
    }
    __syncthreads();
    // sum_k e[j][which][k] * w[k][o], k ascending, 8 weight loads in flight
    auto skinny = [&](const float* __restrict__ w, int K2, int which, int o, float (&acc)[kBiasRays]) {
        int k = 0;
        for (; k + 8 <= K2; k += 8) {
            float wv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) wv[u] = w[(int64_t)(k + u) * nout + o];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int j = 0; j < kBiasRays; ++j) acc[j] = fmaf(e[j][which][k + u], wv[u], acc[j]);
        }
        for (; k < K2; ++k) {
            const float wv = w[(int64_t)k * nout + o];
#pragma unroll
            for (int j = 0; j < kBiasRays; ++j) acc[j] = fmaf(e[j][which][k], wv, acc[j]);
        }
    };
    for (int o = threadIdx.x; o < nout; o += 256) {
        float sd[kBiasRays], st[kBiasRays];
#pragma unroll
        for (int j = 0; j < kBiasRays; ++j) sd[j] = st[j] = 0.0f;
        skinny(wd, 2 * dL, 0, o, sd);
        skinny(wt, 2 * tL, 1, o, st);
#pragma unroll
        for (int j = 0; j < kBiasRays; ++j)
            if (j < nr) bias[(g0 + j) * nout + o] = sd[j] + st[j];
    }
}

}  // namespace

extern "C" int avr_ray_pose_bias(int32_t B, int32_t R, int32_t S, const float* view, const float* tx,
                                 int32_t dir_levels, const void* dir_params, const int64_t* dir_offset,
                                 const float* dir_scale, const int32_t* dir_res, int32_t tx_levels,
                                 const void* tx_params, const int64_t* tx_offset, const float* tx_scale,
                                 const int32_t* tx_res, int32_t param_dtype, int32_t enc_dtype,
                                 int32_t mlp_dtype, const float* w_dir, const float* w_tx, int32_t n_out,
                                 float* bias, void* stream) {
    AVR_REQUIRE(B >= 1 && R >= 1 && S >= 1 && view && tx && dir_params && tx_params && w_dir && w_tx && bias &&
                    n_out >= 1,
                "avr_ray_pose_bias: bad args");
    AVR_REQUIRE(enc_dtype == AVR_DTYPE_F16 || enc_dtype == AVR_DTYPE_F32, "avr_ray_pose_bias: enc dtype");
    AVR_REQUIRE(mlp_dtype == AVR_DTYPE_BF16 || mlp_dtype == AVR_DTYPE_F16, "avr_ray_pose_bias: mlp dtype");
    const int mlp_f16 = mlp_dtype == AVR_DTYPE_F16;
    LevelTable dl, tl;
    if (int e = make_table(dir_levels, dir_offset, dir_scale, dir_res, &dl)) return e;
    if (int e = make_table(tx_levels, tx_offset, tx_scale, tx_res, &tl)) return e;
    const int64_t rays = (int64_t)B * R;
    const dim3 grid((unsigned)((rays + kBiasRays - 1) / kBiasRays));
    const int f16 = enc_dtype == AVR_DTYPE_F16;
    hipStream_t st = as_stream(stream);
    if (param_dtype == AVR_DTYPE_F16)
        hipLaunchKernelGGL(ray_pose_bias_kernel<__half>, grid, dim3(256), 0, st, (int)B, (int)R, (int)S, view, tx,
                           (const __half*)dir_params, dl, (int)dir_levels, (const __half*)tx_params, tl,
                           (int)tx_levels, f16, mlp_f16, w_dir, w_tx, (int)n_out, bias);
    else if (param_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL(ray_pose_bias_kernel<float>, grid, dim3(256), 0, st, (int)B, (int)R, (int)S, view, tx,
                           (const float*)dir_params, dl, (int)dir_levels, (const float*)tx_params, tl,
                           (int)tx_levels, f16, mlp_f16, w_dir, w_tx, (int)n_out, bias);
    else
        return fail(AVR_E_ARG, "avr_ray_pose_bias: unknown param dtype");
    return check_launch("avr_ray_pose_bias");
}
