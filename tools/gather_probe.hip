// Microbenchmark: the fused head's h gather (config 2: h [R=1024][S=256][K=512]
// bf16, 268 MB; a workgroup per (feature group of 64, s) reads 128 B of each
// of the column's 1024 rows, rows in a permuted (delay-sorted) order).
//   mode 1: lane per row, 64-B pieces per lane (the current head_fwd loads)
//   mode 2: 4 lanes per row, one 16-B piece each (quad-coalesced)
//   mode 3: 8 lanes per row, 128 B per row in one instruction
//   mode 0: plain streaming read of the same 268 MB
// Build: hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o tools/_gather_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

constexpr int R = 1024, S = 256, K = 512;
constexpr int ROW16 = K * 2 / 16;  // 16-byte pieces per row (64)
constexpr int KG16 = 8;            // pieces per workgroup per row (128 B)

__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int MODE>
__global__ __launch_bounds__(256) void gather(const uint4* __restrict__ h, const int* __restrict__ perm,
                                              uint32_t* __restrict__ out) {
    const int kg = blockIdx.x, s = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int* pc = perm + s * R;
    uint32_t acc = 0;
    auto row = [&](int r) { return h + ((size_t)r * S + s) * ROW16 + kg * KG16; };
    if constexpr (MODE == 0) {
        const uint4* base = h + ((size_t)(s * 8 + kg)) * (R * ROW16 * S / 2048);
        const int n = R * ROW16 * S / 2048;  // pieces per workgroup
        for (int i = threadIdx.x; i < n; i += 256 * 8) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = base[min(i + u * 256, n - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += fold(v[u]);
        }
    } else if constexpr (MODE == 1) {
        int rr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) rr[u] = pc[threadIdx.x * 4 + u];
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
            uint4 v[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c) v[u][c] = row(rr[u])[sb * 4 + c];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc += fold(v[u][c]);
        }
    } else if constexpr (MODE == 2) {
        const int q = lane >> 2, j = lane & 3;
        int rr[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) rr[m] = pc[wave * 256 + q * 16 + m];
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
            uint4 v[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = row(rr[m])[sb * 4 + j];
#pragma unroll
            for (int m = 0; m < 16; ++m) acc += fold(v[m]);
        }
    } else {
        const int q = lane >> 3, j = lane & 7;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            uint4 v[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = row(pc[wave * 256 + q * 32 + h2 * 16 + m])[j];
#pragma unroll
            for (int m = 0; m < 16; ++m) acc += fold(v[m]);
        }
    }
    out[(blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x] = acc;
}

int main() {
    const size_t nbytes = (size_t)R * S * K * 2;
    uint4* h;
    int* perm;
    uint32_t* out;
    hipMalloc(&h, nbytes);
    hipMemset(h, 1, nbytes);
    hipMalloc(&perm, sizeof(int) * R * S);
    hipMalloc(&out, sizeof(uint32_t) * 8 * S * 256);
    std::mt19937 rng(1);
    std::vector<int> p(R * S);
    for (int pass = 0; pass < 2; ++pass) {
        for (int s = 0; s < S; ++s) {
            for (int r = 0; r < R; ++r) p[s * R + r] = r;
            if (pass == 1) std::shuffle(p.begin() + s * R, p.begin() + (s + 1) * R, rng);
        }
        hipMemcpy(perm, p.data(), sizeof(int) * R * S, hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int mode = 0; mode < 4; ++mode) {
            auto go = [&] {
                dim3 grid(8, S);
                if (mode == 0) gather<0><<<grid, 256>>>(h, perm, out);
                if (mode == 1) gather<1><<<grid, 256>>>(h, perm, out);
                if (mode == 2) gather<2><<<grid, 256>>>(h, perm, out);
                if (mode == 3) gather<3><<<grid, 256>>>(h, perm, out);
            };
            for (int i = 0; i < 5; ++i) go();
            hipEventRecord(e0);
            const int n = 30;
            for (int i = 0; i < n; ++i) go();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / n;
            printf("{\"perm\": \"%s\", \"mode\": %d, \"us\": %.2f, \"TBps\": %.3f}\n", pass ? "random" : "identity", mode,
                   us, nbytes / us / 1e6);
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    return 0;
}
