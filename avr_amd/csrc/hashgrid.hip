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

#include <algorithm>

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
constexpr int64_t kLevelMajorMinPoints = 16384;
inline int64_t lm_min_points() { return kLevelMajorMinPoints; }

// grouped corner loads in the level-major forward (fp16 tables, §9b)
inline bool group_loads() { return true; }

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
                                                              LevelTable lt, To* __restrict__ out, int unit) {
    const int l = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    float xi[3] = {x[i * 3 + 0], x[i * 3 + 1], x[i * 3 + 2]};
    if (unit) {  // (x + 1) / 2 as 0.5 + 0.5 x: the halving is exact, one rounding (model.py:187-189)
#pragma unroll
        for (int d = 0; d < 3; ++d) xi[d] = 0.5f + 0.5f * xi[d];
    }
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
// Each 16-lane group walks RUN consecutive points in order (the renderer's
// points are ray-major, so these are consecutive samples of one ray) and a
// lane keeps a pending (dword, sum): while the next point's corner hits the
// same dword (a coarse cell several samples long) the value is added in
// registers, and only a change of dword, or the end of the walk, issues the
// atomic.  Coarse levels, where up to ~8 samples share a cell, then issue a
// fraction of the requests; fine levels issue one per point as before.  All
// coordinate and gradient loads of the walk are issued up front; the atomics
// need no return, so the walk never waits on them.
template <typename Tg, int RUN>
__global__ __launch_bounds__(256) void hashgrid_bwd_kernel(int64_t N, int L, int l0,
                                                           const float* __restrict__ x,
                                                           const Tg* __restrict__ gout,
                                                           LevelTable lt,
                                                           float* __restrict__ gparams) {
    const int l = l0 + (int)blockIdx.y;
    const int slot = threadIdx.x & 15;
    const int k = slot >> 1, f = slot & 1;
    const int64_t first = ((int64_t)blockIdx.x * 16 + (threadIdx.x >> 4)) * RUN;
    const uint32_t size = (uint32_t)(lt.offset[l + 1] - lt.offset[l]);
    const uint32_t res = lt.res[l];
    const float scale = lt.scale[l];
    float* __restrict__ table = gparams + 2 * lt.offset[l];
    float xi[RUN][3], g[RUN];
#pragma unroll
    for (int it = 0; it < RUN; ++it) {
        const int64_t i = first + it;
        const int64_t ic = i < N ? i : N - 1;
#pragma unroll
        for (int d = 0; d < 3; ++d) xi[it][d] = x[ic * 3 + d];
        g[it] = i < N ? load_f(gout, ic * (2 * L) + 2 * l + f) : 0.0f;
    }
    uint32_t pe = 0xffffffffu;
    float pv = 0.0f;
#pragma unroll
    for (int it = 0; it < RUN; ++it) {
        const Corner c = locate(xi[it], scale);
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
        const float v = wgt * g[it];
        if (e == pe) {
            pv += v;
        } else {
            if (pv != 0.0f) atomicAdd(table + pe, pv);
            pe = e;
            pv = v;
        }
    }
    if (pv != 0.0f) atomicAdd(table + pe, pv);
}

// points walked per 16-lane group
inline int bwd_run() { return 16; }

template <typename Tg>
void launch_bwd(hipStream_t st, int64_t N, int L, const float* x, const Tg* gout, const LevelTable& lt,
                float* gparams) {
    const int run = bwd_run();
    const int64_t pts_per_block = 16 * (int64_t)run;  // 16 groups of 16 lanes
    const dim3 grid((unsigned)((N + pts_per_block - 1) / pts_per_block), (unsigned)L);
#define AVR_HG_BWD(I)                                                                                          \
    if (run == I) {                                                                                            \
        hipLaunchKernelGGL((hashgrid_bwd_kernel<Tg, I>), grid, dim3(256), 0, st, N, L, 0, x, gout, lt, gparams); \
        return;                                                                                                \
    }
    AVR_HG_BWD(1) AVR_HG_BWD(4) AVR_HG_BWD(8) AVR_HG_BWD(16) AVR_HG_BWD(32)
#undef AVR_HG_BWD
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
               void* out, bool grp, int unit) {
    if constexpr (std::is_same_v<Tp, __half>) {
        if (grp) {
            hipLaunchKernelGGL((hashgrid_fwd_lm_kernel<Tp, To, ROW_MAJOR, true>), grid, dim3(256), 0, st, N,
                               x, (const Tp*)params, lt, (To*)out, unit);
            return;
        }
    }
    hipLaunchKernelGGL((hashgrid_fwd_lm_kernel<Tp, To, ROW_MAJOR, false>), grid, dim3(256), 0, st, N, x,
                           (const Tp*)params, lt, (To*)out, unit);
}

// Level-major forward launch; grouped corner loads for fp16 tables whose
// base is 16-byte aligned (level offsets are multiples of 8 entries).  fp32
// tables keep the 8-byte loads: a 16-byte group holds only 2 entries there
// and measured slower (config-2 points: 102 -> 119 us level-major, 141 ->
// 156 us row-major); fp16: 113-117 -> 103-106 us level-major, 138-140 ->
// 116-118 us row-major (profiles/r02_hashgrid_group_ab.jsonl)
template <bool ROW_MAJOR>
int launch_fwd_lm(dim3 grid, hipStream_t st, int64_t N, const float* x, const void* params,
                  int32_t param_dtype, const LevelTable& lt, void* out, int32_t out_dtype, int unit = 0) {
    const bool grp = group_loads() && ((uintptr_t)params & 15) == 0;
    if (param_dtype == AVR_DTYPE_F32 && out_dtype == AVR_DTYPE_F32)
        launch_lm<float, float, ROW_MAJOR>(grid, st, N, x, params, lt, out, grp, unit);
    else if (param_dtype == AVR_DTYPE_F32 && out_dtype == AVR_DTYPE_F16)
        launch_lm<float, __half, ROW_MAJOR>(grid, st, N, x, params, lt, out, grp, unit);
    else if (param_dtype == AVR_DTYPE_F16 && out_dtype == AVR_DTYPE_F16)
        launch_lm<__half, __half, ROW_MAJOR>(grid, st, N, x, params, lt, out, grp, unit);
    else if (param_dtype == AVR_DTYPE_F16 && out_dtype == AVR_DTYPE_F32)
        launch_lm<__half, float, ROW_MAJOR>(grid, st, N, x, params, lt, out, grp, unit);
    else
        return fail(AVR_E_ARG, "avr_hashgrid_fwd: unknown dtype");
    return 0;
}

// ------------------------------------------- partitioned backward (no atomics)
// The atomic backward above is bound by memory-side atomic requests (one per
// 64-B segment a wave-instruction touches, ~4.5 per point and hashed level)
// and, on the coarse levels, by many adders per address (every ray starts at
// the listener, so its first samples share cells at every coarse level).
// This form never adds into HBM concurrently:
//   1. count:   every (level, chunk of kChunkPts points) block walks its
//               points, merges equal entries along each 8-lane group's run,
//               and counts the merged contributions per table partition
//               (kPartEntries consecutive entries of one level) in LDS;
//   2. scan:    one wave per partition turns its per-chunk counts into
//               offsets and a total;
//   3. scatter: the same walk writes each contribution (entry within the
//               partition, value pair) into its partition's segment of a
//               workspace (partition-contiguous, chunk-ordered segments,
//               slot order within a chunk free), staged in LDS by partition
//               so the stores are coalesced;
//   4. reduce:  one wave per partition slice sums its contributions into
//               an LDS image of the partition and adds the image to the
//               gradient with plain vector loads/stores (the wave owns those
//               entries).
// The workspace holds N * L * 8 contributions at most (12 B each).  Both
// walks read the upstream gradient level-major (glm, transposed by its own
// pass first).
constexpr int kPartBits = 10;
constexpr int kPartEntries = 1 << kPartBits;      // 1024 entries = 8 KB of fp32 pairs (one wave's image)
constexpr int kBwdGroups = 32;                    // 8-lane groups per 256-thread block
constexpr int kBwdRun = 16;                       // consecutive points walked per group
constexpr int kChunkPts = kBwdGroups * kBwdRun;   // 512 points per block and level
constexpr int kReduceWaves = 4;                   // reduce block: one partition slice per wave
constexpr int kMaxScatterParts = 4096;            // partitions per level the count/scatter LDS holds

struct BwdPlan {
    int pbase[kMaxLevels + 1];  // first partition of each level (prefix of ceil(size / kPartEntries))
    int nchunks;
    int max_parts;              // partitions of the largest level
    int slice_cap[kMaxLevels];  // contributions per reduce slice ...
    int hot_above[kMaxLevels];  // ... and kDenseSlice for partitions holding more than this (hot cells)
};

// One point's contribution to corner k (the walk's arithmetic): the entry
// and the value pair w_k * g.
__device__ __forceinline__ void corner_value(const float (&xi)[3], float g0, float g1, int k, float scale,
                                             uint32_t size, uint32_t res, uint32_t& e, float& v0, float& v1) {
    const Corner c = locate(xi, scale);
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
    e = grid_index(size, res, gg[0], gg[1], gg[2]);
    v0 = wgt * g0;
    v1 = wgt * g1;
}

// The count and scatter walks read the upstream gradient level-major, glm
// [L][N][2] (hg_level_major_kernel): a block's 512 points of one level are
// 4 KiB of consecutive pairs instead of one 8-byte pair in every 160-byte
// row of grad_out [N][L][2] (a cache line per point and level, twice).
__device__ __forceinline__ int64_t glm_index(int64_t i, int64_t N, int l) { return ((int64_t)l * N + i) * 2; }

// point i's coordinates and level-l gradient pair (zero past N; the walk's
// clamped loads)
template <typename Tg>
__device__ __forceinline__ void point_inputs(int64_t i, int64_t N, int L, int l, const float* __restrict__ x,
                                             const Tg* __restrict__ glm, float (&xi)[3], float& g0, float& g1) {
    const bool live = i < N;
    const int64_t ic = live ? i : N - 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) xi[d] = x[ic * 3 + d];
    const int64_t gi = glm_index(ic, N, l);
    g0 = live ? load_f(glm, gi) : 0.0f;
    g1 = live ? load_f(glm, gi + 1) : 0.0f;
}

// grad_out [N][L][2] -> glm [L][N][2], 64 points per block through LDS
template <typename Tg>
__global__ __launch_bounds__(256) void hg_level_major_kernel(int64_t N, int L, const Tg* __restrict__ in,
                                                             Tg* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char lm_s[];
    Tg* t = reinterpret_cast<Tg*>(lm_s);  // [64][2L]
    const int64_t i0 = (int64_t)blockIdx.x * 64;
    const int np = (int)min((int64_t)64, N - i0);
    const int W = 2 * L;
    for (int j = threadIdx.x; j < np * W; j += 256) t[j] = in[i0 * W + j];
    __syncthreads();
    for (int j = threadIdx.x; j < L * np * 2; j += 256) {
        const int l = j / (np * 2), r = j - l * (np * 2);
        out[((int64_t)l * N + i0) * 2 + r] = t[(r >> 1) * W + 2 * l + (r & 1)];
    }
}

// The walk shared by the count and scatter passes: lane k of 8-lane group g
// owns corner k of the group's kBwdRun consecutive points (both features);
// emit(entry, v0, v1) is called for every merged contribution, in walk order.
template <typename Tg, class Emit>
__device__ __forceinline__ void bwd_walk(int64_t N, int L, int l, const float* __restrict__ x,
                                         const Tg* __restrict__ gout, const LevelTable& lt, Emit&& emit) {
    const int k = threadIdx.x & 7;
    const int64_t first = ((int64_t)blockIdx.x * kBwdGroups + (threadIdx.x >> 3)) * kBwdRun;
    const uint32_t size = (uint32_t)(lt.offset[l + 1] - lt.offset[l]);
    const uint32_t res = lt.res[l];
    const float scale = lt.scale[l];
    float xi[kBwdRun][3], g0[kBwdRun], g1[kBwdRun];
#pragma unroll
    for (int it = 0; it < kBwdRun; ++it) point_inputs(first + it, N, L, l, x, gout, xi[it], g0[it], g1[it]);
    uint32_t pe = 0xffffffffu;
    float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
    for (int it = 0; it < kBwdRun; ++it) {
        uint32_t e;
        float v0, v1;
        corner_value(xi[it], g0[it], g1[it], k, scale, size, res, e, v0, v1);
        if (e == pe) {
            p0 += v0;
            p1 += v1;
        } else {
            if (pe != 0xffffffffu && (p0 != 0.0f || p1 != 0.0f)) emit(pe, p0, p1);
            pe = e;
            p0 = v0;
            p1 = v1;
        }
    }
    if (pe != 0xffffffffu && (p0 != 0.0f || p1 != 0.0f)) emit(pe, p0, p1);
}

template <typename Tg>
__global__ __launch_bounds__(256) void hg_bwd_count_kernel(int64_t N, int L, const float* __restrict__ x,
                                                           const Tg* __restrict__ gout, LevelTable lt,
                                                           BwdPlan plan, int* __restrict__ counts) {
    extern __shared__ int cnt_l[];
    const int l = blockIdx.y;
    const int P = plan.pbase[l + 1] - plan.pbase[l];
    for (int p = threadIdx.x; p < P; p += 256) cnt_l[p] = 0;
    __syncthreads();
    bwd_walk(N, L, l, x, gout, lt,
             [&](uint32_t e, float, float) { atomicAdd(&cnt_l[e >> kPartBits], 1); });
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += 256)
        counts[(int64_t)(plan.pbase[l] + p) * plan.nchunks + blockIdx.x] = cnt_l[p];
}

// one wave per partition: per-chunk counts -> exclusive offsets within the
// partition (in place), and the partition's total
__global__ __launch_bounds__(1024) void hg_bwd_scan_kernel(int total_parts, int nchunks, int* __restrict__ counts,
                                                           int* __restrict__ totals) {
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.x * 16 + (threadIdx.x >> 6);
    if (p >= total_parts) return;
    int* c = counts + (int64_t)p * nchunks;
    int carry = 0;
    for (int c0 = 0; c0 < nchunks; c0 += 64) {
        const int v = c0 + lane < nchunks ? c[c0 + lane] : 0;
        int incl = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(incl, off, 64);
            if (lane >= off) incl += o;
        }
        if (c0 + lane < nchunks) c[c0 + lane] = carry + incl - v;
        carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) totals[p] = carry;
}

// one block: partition starts (exclusive prefix of the totals) and the
// reduce pass's slices.  Every ray of a batch starts at its listener, so on
// the dense (coarse) levels a few cells collect contributions from hundreds
// of rays; their partitions are cut into slices of kDenseSlice contributions
// (each summed by its own wave, the slices then added with no-return
// atomics), so no single wave serialises a hot cell's repeats.  Hashed
// levels keep one slice per partition where possible (plain flush).
constexpr int kDenseSlice = 1024;
// tag rounds before the per-key wave sums take over (a round costs about as
// much as one key's wave sum and serves every distinct key at once: near the
// listener a wave-load holds ~25 keys repeated up to ~7 times)
constexpr int kTagRounds = 4;
constexpr int kHashedSlice = 16384;

// (the plan's level tables in LDS and each thread's totals loaded eight at a
// time, independent of each other: read from the kernel argument with a
// per-thread level index and one total per dependent step, this one-block
// pass took ~12 us per grid)
__global__ __launch_bounds__(1024) void hg_bwd_plan_kernel(int total_parts, BwdPlan plan,
                                                           const int* __restrict__ totals,
                                                           int* __restrict__ part_start,
                                                           int* __restrict__ slice_base) {
    __shared__ int ws_t[16], ws_s[16];
    __shared__ int pbase_s[kMaxLevels + 1], hot_s[kMaxLevels], cap_s[kMaxLevels];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x <= kMaxLevels) pbase_s[threadIdx.x] = plan.pbase[threadIdx.x];
    if (threadIdx.x < kMaxLevels) {
        hot_s[threadIdx.x] = plan.hot_above[threadIdx.x];
        cap_s[threadIdx.x] = plan.slice_cap[threadIdx.x];
    }
    __syncthreads();
    // thread t owns the `per` consecutive partitions from per * t: one
    // block-wide scan for all of them
    const int per = (total_parts + 1 + 1023) / 1024;
    const int q0 = threadIdx.x * per;
    int l0 = 0;
    while (l0 < kMaxLevels && pbase_s[l0 + 1] <= q0) ++l0;
    // the slices partition q's total t takes
    auto slices = [&](int t, int l) {
        const int cap = t > hot_s[l] ? kDenseSlice : cap_s[l];
        return max(1, (t + cap - 1) / cap);
    };
    int st = 0, ss = 0;  // this thread's sums
    int l = l0;
    for (int j0 = 0; j0 < per; j0 += 8) {
        int tv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + j0 + u;
            tv[u] = (j0 + u < per && q < total_parts) ? totals[q] : -1;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (tv[u] < 0) break;
            const int q = q0 + j0 + u;
            while (pbase_s[l + 1] <= q) ++l;
            st += tv[u];
            ss += slices(tv[u], l);
        }
    }
    int it = st, is = ss;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int ut = __shfl_up(it, off, 64), us = __shfl_up(is, off, 64);
        if (lane >= off) {
            it += ut;
            is += us;
        }
    }
    if (lane == 63) {
        ws_t[wave] = it;
        ws_s[wave] = is;
    }
    __syncthreads();
    int pt = 0, ps = 0;
    for (int w = 0; w < wave; ++w) {
        pt += ws_t[w];
        ps += ws_s[w];
    }
    int rt = pt + it - st, rs = ps + is - ss;  // exclusive prefixes at q0
    l = l0;
    for (int j0 = 0; j0 < per; j0 += 8) {
        int tv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + j0 + u;
            tv[u] = (j0 + u < per && q < total_parts) ? totals[q] : -1;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + j0 + u;
            if (j0 + u >= per || q > total_parts) break;
            part_start[q] = rt;
            slice_base[q] = rs;
            if (q == total_parts) break;
            while (pbase_s[l + 1] <= q) ++l;
            rt += tv[u];
            rs += slices(tv[u], l);
        }
    }
}

// The scatter walk stages the block's merged contributions in LDS, grouped
// by partition at block-local offsets (the scan of its own counts), and then
// copies them out in staged order: consecutive lanes store consecutive
// records of one partition's segment.  Stored straight from the walk, each
// lane's 12 bytes went to another partition's segment: one cache line per
// lane and store instruction (issue-bound), and partly written lines
// (written back as ~1.5x the record bytes).  The staged record carries its
// partition in the key's upper bits.
constexpr int kScatMaxRecs = 256 * kBwdRun;  // merged contributions of one block at most
static_assert(((int64_t)kMaxScatterParts << kPartBits) <= (int64_t(1) << 32), "staged key: partition + entry in 32 bits");
static_assert((3 * kScatMaxRecs + 3 * kMaxScatterParts + 1) * 4 + 16 <= 160 * 1024, "scatter LDS");

template <typename Tg>
__global__ __launch_bounds__(256) void hg_bwd_scatter_kernel(int64_t N, int L, const float* __restrict__ x,
                                                             const Tg* __restrict__ gout, LevelTable lt,
                                                             BwdPlan plan, const int* __restrict__ offs,
                                                             const int* __restrict__ totals,
                                                             const int* __restrict__ part_start,
                                                             uint3* __restrict__ contrib) {
    extern __shared__ __attribute__((aligned(16))) int scat_l[];  // stage[3 kScatMaxRecs], base[P], lofs[P + 1], slot[P]
    __shared__ int wsum[4];
    const int l = blockIdx.y;
    const int pb = plan.pbase[l];
    const int P = plan.pbase[l + 1] - pb;
    uint32_t* stage = reinterpret_cast<uint32_t*>(scat_l);
    int* base = scat_l + 3 * kScatMaxRecs;
    int* lofs = base + P;
    int* slot = lofs + P + 1;
    const int chunk = blockIdx.x, nch = plan.nchunks;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // this chunk's count and global segment start per partition (the scan
    // pass left exclusive offsets within each partition); E consecutive
    // partitions per thread
    const int E = (P + 255) / 256;
    const int q0 = threadIdx.x * E;
    int run = 0;
    for (int j = 0; j < E; ++j) {
        const int q = q0 + j;
        if (q >= P) break;
        const int64_t at = (int64_t)(pb + q) * nch + chunk;
        const int o = offs[at];
        const int c = (chunk + 1 < nch ? offs[at + 1] : totals[pb + q]) - o;
        base[q] = part_start[pb + q] + o;
        slot[q] = 0;
        lofs[q] = c;  // (the count, until the scan below)
        run += c;
    }
    int incl = run;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int acc = incl - run;
    for (int w = 0; w < wave; ++w) acc += wsum[w];
    for (int j = 0; j < E; ++j) {
        const int q = q0 + j;
        if (q >= P) break;
        const int c = lofs[q];
        lofs[q] = acc;
        acc += c;
    }
    if (threadIdx.x == 0) lofs[P] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    bwd_walk(N, L, l, x, gout, lt, [&](uint32_t e, float v0, float v1) {
        const int part = (int)(e >> kPartBits);
        const int lp = lofs[part] + atomicAdd(&slot[part], 1);
        stage[3 * lp] = ((uint32_t)part << kPartBits) | (e & (kPartEntries - 1));
        stage[3 * lp + 1] = __float_as_uint(v0);
        stage[3 * lp + 2] = __float_as_uint(v1);
    });
    __syncthreads();
    const int total = lofs[P];
    for (int r = threadIdx.x; r < total; r += 256) {
        const uint32_t s0 = stage[3 * r], s1 = stage[3 * r + 1], s2 = stage[3 * r + 2];
        const int q = (int)(s0 >> kPartBits);
        // one 12-byte store per contribution: (key, v0, v1)
        contrib[base[q] + (r - lofs[q])] = make_uint3(s0 & (kPartEntries - 1), s1, s2);
    }
}

// Sum of x over the wave, uniform (DPP within rows of 16, then the four row
// sums read as scalars: no LDS round trip, unlike __shfl_xor)
template <int C>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), C, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_total(float x) {
    x += dpp_f<0xB1>(x);   // quad_perm [1,0,3,2]
    x += dpp_f<0x4E>(x);   // quad_perm [2,3,0,1]
    x += dpp_f<0x141>(x);  // row_half_mirror
    x += dpp_f<0x140>(x);  // row_mirror
    const int xi = __float_as_int(x);
    return (__int_as_float(__builtin_amdgcn_readlane(xi, 0)) + __int_as_float(__builtin_amdgcn_readlane(xi, 16))) +
           (__int_as_float(__builtin_amdgcn_readlane(xi, 32)) + __int_as_float(__builtin_amdgcn_readlane(xi, 48)));
}

// One wave per partition slice, with the partition's image in the wave's own
// LDS (no other wave touches it).  LDS float atomics measured slow on this
// path (the reduce pass took ~160 of 330 us with ds_add_f32), so each
// contribution is added with a plain read-add-write, made safe by a tag
// round: every pending lane writes its lane id into tag[key], reads it back,
// and only the lanes that find their own id add (their keys are distinct);
// the others are summed per key across the wave and added once per key.
// Keys repeat within one wave-load only where many rays cross the same
// cells (coarse levels), so the tag round alone is the rule.
__global__ __launch_bounds__(64 * kReduceWaves) void hg_bwd_reduce_kernel(LevelTable lt, BwdPlan plan, int total_parts,
                                                                         const int* __restrict__ totals,
                                                                         const int* __restrict__ part_start,
                                                                         const int* __restrict__ slice_base,
                                                                         const uint3* __restrict__ contrib,
                                                                         float* __restrict__ gparams, int overwrite) {
    __shared__ float2 img_all[kReduceWaves][kPartEntries];
    __shared__ uint8_t tag_all[kReduceWaves][kPartEntries];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float2* img = img_all[wave];
    uint8_t* tag = tag_all[wave];
    const int b = blockIdx.x * kReduceWaves + wave;
    if (b >= slice_base[total_parts]) return;  // the grid is sized for the worst case
    // partition p: slice_base[p] <= b < slice_base[p + 1]
    int lo = 0, hi = total_parts - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (slice_base[mid] <= b) lo = mid; else hi = mid - 1;
    }
    const int p = lo;
    const int ns = slice_base[p + 1] - slice_base[p], sl = b - slice_base[p];
    const int n = totals[p];
    int l = 0;
    while (plan.pbase[l + 1] <= p) ++l;
    const int64_t e0 = (int64_t)(p - plan.pbase[l]) * kPartEntries;
    // level sizes are multiples of 8 entries: ne is, and the partition's
    // 2*ne floats start 16-byte aligned
    const int ne = (int)min((int64_t)kPartEntries, lt.offset[l + 1] - lt.offset[l] - e0);
    float* dstf = gparams + 2 * (lt.offset[l] + e0);
    if (n == 0) {  // wave-uniform
        if (overwrite) {  // (a partition without contributions has one slice)
            float4* dst = reinterpret_cast<float4*>(dstf);
            for (int i = lane; i < ne / 2; i += 64) dst[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        return;
    }
    const int i0 = part_start[p] + (int)((int64_t)n * sl / ns);
    const int i1 = part_start[p] + (int)((int64_t)n * (sl + 1) / ns);
    for (int i = lane; i < ne; i += 64) img[i] = make_float2(0.f, 0.f);
    constexpr int U = 8;
    for (int i = i0; i < i1; i += 64 * U) {
        uint32_t kk[U];
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = i + 64 * u + lane;
            const uint3 cv = contrib[j < i1 ? j : i0];
            kk[u] = j < i1 ? cv.x : 0u;
            v[u] = j < i1 ? make_float2(__uint_as_float(cv.y), __uint_as_float(cv.z)) : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            bool todo = i + 64 * u + lane < i1;
            // up to kTagRounds rounds: each adds one lane per distinct pending key
            for (int round = 0; round < kTagRounds; ++round) {
                if (todo) tag[kk[u]] = (uint8_t)lane;
                // compiler barrier: the read-back must not be folded into the
                // lane's own write (LDS keeps one wave's accesses in order)
                asm volatile("" ::: "memory");
                // the image entry is read with the tag (one wait, not two):
                // only this round's winner for a key writes it, after the read
                int tg = -1;
                float2 a = make_float2(0.f, 0.f);
                if (todo) {
                    tg = tag[kk[u]];
                    a = img[kk[u]];
                }
                // (keeps hipcc from sinking the image read into the branch)
                asm volatile("" ::"v"(tg), "v"(a.x), "v"(a.y));
                if (todo && tg == lane) {
                    a.x += v[u].x;
                    a.y += v[u].y;
                    img[kk[u]] = a;
                    todo = false;
                }
                asm volatile("" ::: "memory");
                if (!__ballot(todo)) break;
            }
            // lanes whose key another lane of this load also holds: sum each
            // such key's values across the wave (DPP sums) and add once.
            // One iteration per distinct repeated key: none on the hashed
            // levels as a rule, a few where many rays cross one coarse cell
            uint64_t rest = __ballot(todo);
            while (rest) {
                const int first = __ffsll((unsigned long long)rest) - 1;
                const uint32_t lead = (uint32_t)__builtin_amdgcn_readlane((int)kk[u], first);
                const bool mine = todo && kk[u] == lead;
                const float s0 = wave_total(mine ? v[u].x : 0.0f);
                const float s1 = wave_total(mine ? v[u].y : 0.0f);
                if (lane == first) {
                    float2 a = img[lead];
                    a.x += s0;
                    a.y += s1;
                    img[lead] = a;
                }
                asm volatile("" ::: "memory");
                todo = todo && !mine;
                rest = __ballot(todo);
            }
        }
    }
    const float4* img4 = reinterpret_cast<const float4*>(img);
    if (ns == 1) {  // the wave owns these entries: plain read-add-write (or write)
        float4* dst = reinterpret_cast<float4*>(dstf);
        for (int i = lane; i < ne / 2; i += 64) {
            float4 a = overwrite ? make_float4(0.f, 0.f, 0.f, 0.f) : dst[i];
            const float4 c = img4[i];
            a.x += c.x;
            a.y += c.y;
            a.z += c.z;
            a.w += c.w;
            dst[i] = a;
        }
    } else {  // several slices: no-return atomics of the touched entries
        // (overwrite: hg_bwd_zero_hot_kernel cleared these partitions first)
        const float* imgf = reinterpret_cast<const float*>(img);
        for (int i = lane; i < 2 * ne; i += 64)
            if (imgf[i] != 0.0f) atomicAdd(dstf + i, imgf[i]);
    }
}

// overwrite form: the partitions the reduce splits over several slices
// (their slices add with atomics) are cleared first; one block per partition
__global__ __launch_bounds__(256) void hg_bwd_zero_hot_kernel(LevelTable lt, BwdPlan plan, int total_parts,
                                                              const int* __restrict__ slice_base,
                                                              float* __restrict__ gparams) {
    const int p = blockIdx.x;
    if (p >= total_parts || slice_base[p + 1] - slice_base[p] <= 1) return;
    int l = 0;
    while (plan.pbase[l + 1] <= p) ++l;
    const int64_t e0 = (int64_t)(p - plan.pbase[l]) * kPartEntries;
    const int ne = (int)min((int64_t)kPartEntries, lt.offset[l + 1] - lt.offset[l] - e0);
    float4* dst = reinterpret_cast<float4*>(gparams + 2 * (lt.offset[l] + e0));
    for (int i = threadIdx.x; i < ne / 2; i += 256) dst[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

constexpr int64_t kMaxBwdWorkspaceBytes = int64_t(1) << 31;  // 2 GiB (config 4: 283 MB)

struct BwdLayout {
    BwdPlan plan;
    int total_parts;
    int64_t counts, totals, part_start, slice_base, glm, contrib, bytes;  // byte offsets in the workspace
    int max_slices;  // reduce grid: total_parts + maxc / kDenseSlice bounds the slice count
    bool scatter_ok; // the largest level's partition table fits the count/scatter LDS
};

int bwd_layout(int64_t N, int L, const int64_t* off, const int32_t* res, BwdLayout* o) {
    if (L < 1 || L > kMaxLevels) return fail(AVR_E_ARG, "hashgrid: n_levels out of range (1..32)");
    BwdLayout b{};
    bool res_dense[kMaxLevels];
    for (int l = 0; l < L; ++l) {  // dense level: the grid fits the table (grid_index's rule)
        const double cells = res ? (double)res[l] * res[l] * res[l] : 1e300;
        res_dense[l] = cells <= (double)(off[l + 1] - off[l]);
    }
    b.plan.pbase[0] = 0;
    b.plan.max_parts = 0;
    for (int l = 0; l < L; ++l) {
        const int64_t size = off[l + 1] - off[l];
        if (size <= 0 || size % 8) return fail(AVR_E_ARG, "hashgrid: level sizes must be positive multiples of 8");
        const int64_t P = (size + kPartEntries - 1) / kPartEntries;
        if (b.plan.pbase[l] + P > (1 << 24)) return fail(AVR_E_ARG, "hashgrid: tables too large");
        b.plan.pbase[l + 1] = b.plan.pbase[l] + (int)P;
        // a hashed level spreads N * 8 contributions over its partitions; one
        // holding 1.5x its share has hot cells.  Dense levels are hot by nature
        b.plan.slice_cap[l] = res_dense[l] ? kDenseSlice : kHashedSlice;
        const double share = (double)N * 8.0 * (double)std::min<int64_t>(size, kPartEntries) / (double)size;
        b.plan.hot_above[l] = res_dense[l] ? 0 : (int)std::min(1.5 * share + 64.0, 2.0e9);
        b.plan.max_parts = std::max(b.plan.max_parts, (int)P);
    }
    const int64_t nchunks = (N + kChunkPts - 1) / kChunkPts;
    const int64_t maxc = N * L * 8;
    if (maxc >= (int64_t(1) << 31) || nchunks > 65535)
        return fail(AVR_E_ARG, "hashgrid: too many points for the partitioned backward");
    b.plan.nchunks = (int)std::max<int64_t>(nchunks, 1);
    b.total_parts = b.plan.pbase[L];
    auto al = [](int64_t v) { return (v + 255) & ~(int64_t)255; };
    int64_t o0 = 0;
    b.counts = o0;
    o0 += al((int64_t)b.total_parts * b.plan.nchunks * 4);
    b.totals = o0;
    o0 += al((int64_t)b.total_parts * 4);
    b.part_start = o0;
    o0 += al((int64_t)(b.total_parts + 1) * 4);
    b.slice_base = o0;
    o0 += al((int64_t)(b.total_parts + 1) * 4);
    b.max_slices = b.total_parts + (int)(maxc / kDenseSlice) + 1;
    b.scatter_ok = b.plan.max_parts <= kMaxScatterParts;
    b.glm = o0;  // the upstream gradient level-major (fp32 or fp16: sized for fp32)
    o0 += al(N * L * 2 * 4);
    b.contrib = o0;  // (key, v0, v1) per contribution
    o0 += al(maxc * 12);
    b.bytes = o0;
    // the workspace comes from the caller's allocator on every backward: past
    // this size the atomic kernel runs instead (no workspace, same += result)
    if (b.bytes > kMaxBwdWorkspaceBytes) b.scatter_ok = false;
    *o = b;
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
    hipStream_t st = as_stream(stream);
    if (grad_dtype == AVR_DTYPE_F32)
        launch_bwd<float>(st, N, (int)n_levels, x, (const float*)grad_out, lt, grad_params);
    else if (grad_dtype == AVR_DTYPE_F16)
        launch_bwd<__half>(st, N, (int)n_levels, x, (const __half*)grad_out, lt, grad_params);
    else
        return fail(AVR_E_ARG, "avr_hashgrid_bwd: unknown grad dtype");
    return check_launch("avr_hashgrid_bwd");
}

namespace {
int fwd_lm(int64_t N, int32_t n_levels, const float* x, const void* params, int32_t param_dtype,
           const int64_t* level_offset, const float* level_scale, const int32_t* level_res, void* out,
           int32_t out_dtype, void* stream, int unit) {
    AVR_REQUIRE(N >= 0 && x && params && level_offset && level_scale && level_res && out,
                "avr_hashgrid_fwd_lm: bad args");
    if (N == 0) return 0;
    LevelTable lt;
    if (int e = make_table(n_levels, level_offset, level_scale, level_res, &lt)) return e;
    const dim3 grid((unsigned)((N + 255) / 256), (unsigned)n_levels);
    hipStream_t st = as_stream(stream);
    if (int e = launch_fwd_lm<false>(grid, st, N, x, params, param_dtype, lt, out, out_dtype, unit)) return e;
    return check_launch("avr_hashgrid_fwd_lm");
}
}  // namespace

extern "C" int avr_hashgrid_fwd_lm(int64_t N, int32_t n_levels, const float* x, const void* params,
                                   int32_t param_dtype, const int64_t* level_offset,
                                   const float* level_scale, const int32_t* level_res, void* out,
                                   int32_t out_dtype, void* stream) {
    return fwd_lm(N, n_levels, x, params, param_dtype, level_offset, level_scale, level_res, out, out_dtype, stream,
                  0);
}

// The same on points in [-1, 1]: the encoding of (x + 1) / 2 (model.py:187-189),
// the map applied on load instead of by a separate pass over x.
extern "C" int avr_hashgrid_fwd_lm_unit(int64_t N, int32_t n_levels, const float* x, const void* params,
                                        int32_t param_dtype, const int64_t* level_offset,
                                        const float* level_scale, const int32_t* level_res, void* out,
                                        int32_t out_dtype, void* stream) {
    return fwd_lm(N, n_levels, x, params, param_dtype, level_offset, level_scale, level_res, out, out_dtype, stream,
                  1);
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

// Rays of one pose per workgroup (R % kBias2Rays == 0): one output per
// thread (512 threads), the whole k range of that output's weight column in
// flight at once (one L2 round trip per grid instead of one per 8 k), and the
// pose's tx term computed once for the workgroup's rays.  The same fma chains
// (k ascending) and the same final sd + st as ray_pose_bias_kernel: the
// results are equal bit for bit.  4 rays per workgroup: 256 workgroups for
// config 2's 1024 rays (15.6 us; 16.4-16.9 with 8 rays and 128 workgroups).
constexpr int kBias2Rays = 4;
#ifndef AVR_BIAS_V1  // (A/B: 1 keeps the round-4 kernel for every R)
#define AVR_BIAS_V1 0
#endif
constexpr int kBias2Threads = 512;

template <typename Tp>
__global__ __launch_bounds__(kBias2Threads) void ray_pose_bias2_kernel(
    int B, int R, int S, const float* __restrict__ view, const float* __restrict__ tx, const Tp* __restrict__ dp,
    LevelTable dl, int dL, const Tp* __restrict__ tp, LevelTable tl, int tL, int f16, int mlp_f16,
    const float* __restrict__ wd, const float* __restrict__ wt, int nout, float* __restrict__ bias) {
    __shared__ float ed[kBias2Rays][2 * kMaxLevels];
    __shared__ float et[2 * kMaxLevels];
    const int64_t g0 = (int64_t)blockIdx.x * kBias2Rays;  // R % kBias2Rays == 0: one pose
    const int64_t b = g0 / R;
    for (int q = threadIdx.x; q < (kBias2Rays + 1) * kMaxLevels; q += kBias2Threads) {
        const int j = q / kMaxLevels, l = q % kMaxLevels;
        const bool is_tx = j == kBias2Rays;
        if (l >= (is_tx ? tL : dL)) continue;
        const int64_t r = (g0 + j) % R;
        const float* src = is_tx ? tx + b * R * S * 3 : view + (b * R * S + r * S) * 3;
        const float xi[3] = {(src[0] + 1.0f) / 2.0f, (src[1] + 1.0f) / 2.0f, (src[2] + 1.0f) / 2.0f};
        const float2 v = is_tx ? encode_point_level(xi, tp, tl, l) : encode_point_level(xi, dp, dl, l);
        float* e = is_tx ? et : ed[j];
        e[2 * l] = round_feature(v.x, f16, mlp_f16);
        e[2 * l + 1] = round_feature(v.y, f16, mlp_f16);
    }
    __syncthreads();
    for (int o = threadIdx.x; o < nout; o += kBias2Threads) {
        // weight rows 16 at a time, all in flight before their FMAs
        constexpr int KB = 16;
        float st = 0.0f;
        for (int k0 = 0; k0 < 2 * tL; k0 += KB) {
            float w[KB];
#pragma unroll
            for (int u = 0; u < KB; ++u) w[u] = k0 + u < 2 * tL ? wt[(int64_t)(k0 + u) * nout + o] : 0.0f;
#pragma unroll
            for (int u = 0; u < KB; ++u)
                if (k0 + u < 2 * tL) st = fmaf(et[k0 + u], w[u], st);
        }
        float sd[kBias2Rays];
#pragma unroll
        for (int r = 0; r < kBias2Rays; ++r) sd[r] = 0.0f;
        for (int k0 = 0; k0 < 2 * dL; k0 += KB) {
            float w[KB];
#pragma unroll
            for (int u = 0; u < KB; ++u) w[u] = k0 + u < 2 * dL ? wd[(int64_t)(k0 + u) * nout + o] : 0.0f;
#pragma unroll
            for (int u = 0; u < KB; ++u)
                if (k0 + u < 2 * dL)
#pragma unroll
                    for (int r = 0; r < kBias2Rays; ++r) sd[r] = fmaf(ed[r][k0 + u], w[u], sd[r]);
        }
#pragma unroll
        for (int r = 0; r < kBias2Rays; ++r) bias[(g0 + r) * nout + o] = sd[r] + st;
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
    if (R % kBias2Rays == 0 && !AVR_BIAS_V1) {
        const dim3 grid2((unsigned)(rays / kBias2Rays));
        if (param_dtype == AVR_DTYPE_F16)
            hipLaunchKernelGGL(ray_pose_bias2_kernel<__half>, grid2, dim3(kBias2Threads), 0, st, (int)B, (int)R,
                               (int)S, view, tx, (const __half*)dir_params, dl, (int)dir_levels,
                               (const __half*)tx_params, tl, (int)tx_levels, f16, mlp_f16, w_dir, w_tx, (int)n_out,
                               bias);
        else if (param_dtype == AVR_DTYPE_F32)
            hipLaunchKernelGGL(ray_pose_bias2_kernel<float>, grid2, dim3(kBias2Threads), 0, st, (int)B, (int)R,
                               (int)S, view, tx, (const float*)dir_params, dl, (int)dir_levels,
                               (const float*)tx_params, tl, (int)tx_levels, f16, mlp_f16, w_dir, w_tx, (int)n_out,
                               bias);
        else
            return fail(AVR_E_ARG, "avr_ray_pose_bias: unknown param dtype");
        return check_launch("avr_ray_pose_bias");
    }
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

// Below this many points the atomic kernel is cheaper than the five
// partitioned launches (the per-ray and per-pose grids of the training step)
constexpr int64_t kPartitionedMinPoints = 16384;

extern "C" int avr_hashgrid_bwd_workspace(int64_t N, int32_t n_levels, const int64_t* level_offset,
                                          int64_t* bytes) {
    AVR_REQUIRE(N >= 0 && level_offset && bytes, "avr_hashgrid_bwd_workspace: bad args");
    if (N < kPartitionedMinPoints) {
        *bytes = 256;
        return 0;
    }
    if (n_levels < 1 || n_levels > kMaxLevels) return fail(AVR_E_ARG, "hashgrid: n_levels out of range (1..32)");
    BwdLayout b;
    // shapes the partitioned passes do not take (over 2^31 contributions,
    // level sizes not multiples of 8) run the atomic kernel: no workspace
    *bytes = (bwd_layout(N, n_levels, level_offset, nullptr, &b) == 0 && b.scatter_ok) ? b.bytes : 256;
    return 0;
}

namespace {
int bwd_partitioned(int64_t N, int32_t n_levels, const float* x, const void* grad_out, int32_t grad_dtype,
                    const int64_t* level_offset, const float* level_scale, const int32_t* level_res,
                    float* grad_params, void* workspace, int64_t workspace_bytes, void* stream, bool overwrite) {
    AVR_REQUIRE(N >= 0 && x && grad_out && level_offset && level_scale && level_res && grad_params && workspace,
                "avr_hashgrid_bwd_partitioned: bad args");
    AVR_REQUIRE(reinterpret_cast<uintptr_t>(grad_params) % 16 == 0 && reinterpret_cast<uintptr_t>(workspace) % 256 == 0,
                "avr_hashgrid_bwd_partitioned: grad_params must be 16-byte, workspace 256-byte aligned");
    AVR_REQUIRE(grad_dtype == AVR_DTYPE_F32 || grad_dtype == AVR_DTYPE_F16,
                "avr_hashgrid_bwd_partitioned: unknown grad dtype");
    LevelTable lt;
    if (int e = make_table(n_levels, level_offset, level_scale, level_res, &lt)) return e;
    hipStream_t st = as_stream(stream);
    const int L = n_levels;
    // the overwrite form's atomic paths (few points, shapes the partitioned
    // passes do not take) add into a cleared gradient
    auto clear = [&]() -> bool {
        return !overwrite ||
               hipMemsetAsync(grad_params, 0, (size_t)(2 * level_offset[L]) * sizeof(float), st) == hipSuccess;
    };
    if (N == 0) return clear() ? 0 : fail(AVR_E_ARG, "avr_hashgrid_bwd_partitioned_set: clear failed");
    if (N < kPartitionedMinPoints) {  // few points: the atomic kernel (same += result)
        if (!clear()) return fail(AVR_E_ARG, "avr_hashgrid_bwd_partitioned_set: clear failed");
        if (grad_dtype == AVR_DTYPE_F32)
            launch_bwd<float>(st, N, L, x, (const float*)grad_out, lt, grad_params);
        else
            launch_bwd<__half>(st, N, L, x, (const __half*)grad_out, lt, grad_params);
        return check_launch("avr_hashgrid_bwd_partitioned");
    }
    BwdLayout b;
    if (bwd_layout(N, n_levels, level_offset, level_res, &b) != 0 || !b.scatter_ok) {
        // shapes the partitioned passes do not take: the atomic kernel (same += result)
        if (!clear()) return fail(AVR_E_ARG, "avr_hashgrid_bwd_partitioned_set: clear failed");
        if (grad_dtype == AVR_DTYPE_F32)
            launch_bwd<float>(st, N, L, x, (const float*)grad_out, lt, grad_params);
        else
            launch_bwd<__half>(st, N, L, x, (const __half*)grad_out, lt, grad_params);
        return check_launch("avr_hashgrid_bwd_partitioned");
    }
    AVR_REQUIRE(workspace_bytes >= b.bytes, "avr_hashgrid_bwd_partitioned: workspace too small");
    char* ws = static_cast<char*>(workspace);
    int* counts = reinterpret_cast<int*>(ws + b.counts);
    int* totals = reinterpret_cast<int*>(ws + b.totals);
    uint3* contrib = reinterpret_cast<uint3*>(ws + b.contrib);
    const dim3 grid((unsigned)b.plan.nchunks, (unsigned)L);
    const size_t lds_count = (size_t)b.plan.max_parts * 4;
    const size_t lds_scat = (size_t)(3 * kScatMaxRecs + 3 * b.plan.max_parts + 1) * 4;
    // every pass below reads the gradient level-major
    const dim3 tgrid((unsigned)((N + 63) / 64));
    void* glm = ws + b.glm;
    if (grad_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL(hg_level_major_kernel<float>, tgrid, dim3(256), 64 * 2 * L * 4, st, N, L,
                           (const float*)grad_out, (float*)glm);
    else
        hipLaunchKernelGGL(hg_level_major_kernel<__half>, tgrid, dim3(256), 64 * 2 * L * 2, st, N, L,
                           (const __half*)grad_out, (__half*)glm);
    grad_out = glm;
    if (grad_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL(hg_bwd_count_kernel<float>, grid, dim3(256), lds_count, st, N, L, x,
                           (const float*)grad_out, lt, b.plan, counts);
    else
        hipLaunchKernelGGL(hg_bwd_count_kernel<__half>, grid, dim3(256), lds_count, st, N, L, x,
                           (const __half*)grad_out, lt, b.plan, counts);
    int* part_start = reinterpret_cast<int*>(ws + b.part_start);
    int* slice_base = reinterpret_cast<int*>(ws + b.slice_base);
    hipLaunchKernelGGL(hg_bwd_scan_kernel, dim3((unsigned)((b.total_parts + 15) / 16)), dim3(1024), 0, st,
                       b.total_parts, b.plan.nchunks, counts, totals);
    hipLaunchKernelGGL(hg_bwd_plan_kernel, dim3(1), dim3(1024), 0, st, b.total_parts, b.plan, totals, part_start,
                       slice_base);
    if (grad_dtype == AVR_DTYPE_F32)
        hipLaunchKernelGGL(hg_bwd_scatter_kernel<float>, grid, dim3(256), lds_scat, st, N, L, x,
                           (const float*)grad_out, lt, b.plan, counts, totals, part_start, contrib);
    else
        hipLaunchKernelGGL(hg_bwd_scatter_kernel<__half>, grid, dim3(256), lds_scat, st, N, L, x,
                           (const __half*)grad_out, lt, b.plan, counts, totals, part_start, contrib);
    if (overwrite)
        hipLaunchKernelGGL(hg_bwd_zero_hot_kernel, dim3((unsigned)b.total_parts), dim3(256), 0, st, lt, b.plan,
                           b.total_parts, slice_base, grad_params);
    hipLaunchKernelGGL(hg_bwd_reduce_kernel, dim3((unsigned)((b.max_slices + kReduceWaves - 1) / kReduceWaves)),
                       dim3(64 * kReduceWaves), 0, st, lt, b.plan, b.total_parts, totals, part_start, slice_base,
                       contrib, grad_params, (int)overwrite);
    return check_launch("avr_hashgrid_bwd_partitioned");
}
}  // namespace

extern "C" int avr_hashgrid_bwd_partitioned(int64_t N, int32_t n_levels, const float* x, const void* grad_out,
                                            int32_t grad_dtype, const int64_t* level_offset,
                                            const float* level_scale, const int32_t* level_res,
                                            float* grad_params, void* workspace, int64_t workspace_bytes,
                                            void* stream) {
    return bwd_partitioned(N, n_levels, x, grad_out, grad_dtype, level_offset, level_scale, level_res, grad_params,
                           workspace, workspace_bytes, stream, false);
}

// The same gradient written instead of added: grad_params need not be
// cleared first (every entry of every level is written exactly once, zeros
// where no point contributes; the partitions several reduce slices share
// are cleared by their own pass).  Saves the caller's fill of the table
// and the reduce pass's read of it.
extern "C" int avr_hashgrid_bwd_partitioned_set(int64_t N, int32_t n_levels, const float* x, const void* grad_out,
                                                int32_t grad_dtype, const int64_t* level_offset,
                                                const float* level_scale, const int32_t* level_res,
                                                float* grad_params, void* workspace, int64_t workspace_bytes,
                                                void* stream) {
    return bwd_partitioned(N, n_levels, x, grad_out, grad_dtype, level_offset, level_scale, level_res, grad_params,
                           workspace, workspace_bytes, stream, true);
}
