// Loading a wave's stationary MFMA operand (32 rows x 512 16-bit values,
// the A fragments of v_mfma_f32_32x32x16: lane (j, half) holds row j,
// k = 16 ks + 8 half + 0..7) through LDS-DMA (csrc/head_exact.hip,
// csrc/linear_fwd.hip).
//
// Loaded straight into registers, every wave-instruction reads 32 B from each
// of 32 rows: at 256 rows per workgroup that took 16-20 us per work item on
// MI355X (tools/probe_phases.py: 26-43 % of a wave's life), latency-bound on
// the cache lines in flight.  By LDS-DMA every instruction moves one whole
// 1 KiB row, and the fragments are then read from LDS: four rounds of 8
// rows through two 8 KiB buffers per wave, the next round in flight while a
// round is read.
#pragma once

#include "common.h"

namespace avr {

typedef uint32_t frag8_t __attribute__((ext_vector_type(4)));

// One 16-byte-per-lane LDS-DMA load: lane i's 16 bytes at g land at LDS byte
// address lds + 16 i (inline asm: the compiler does not treat the DMA as an
// LDS write that later ds_reads wait for; completion is waited by vmcnt).
// The rows are read once per launch (a work item's rows belong to it alone):
// non-temporal (nt), so they stream past L2 instead of evicting what the
// workgroups re-read from it (the exact head's W tiles, 4 MiB at config 5 =
// one XCD's L2; MI355X_MICROARCH.md "nt-weights": once-read bytes).
__device__ __forceinline__ void stat_dma16(const void* g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(lds), "v"(g)
                 : "memory", "m0");
}

// Rows 8k .. 8k+7 of the wave's 32 (lane j holds row j's base in `row`)
// into staging buffer k & 1 (8 KiB each): one 1 KiB DMA per row, row jr's
// 16-byte chunks rotated by jr slots (the DMA source of lane i is chunk
// (i + jr) mod 64), so the 8 rows one fragment read touches fall on
// distinct banks.
// The lane index through an empty asm: a value the compiler cannot hoist out
// of an enclosing loop, so the per-lane offsets below are formed where they
// are used instead of held in registers across a persistent kernel's loop.
__device__ __forceinline__ int stat_lane() {
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    return lane;
}

__device__ __forceinline__ void stat_issue_round(const uint16_t* row, char* stage, int k) {
    const int lane = stat_lane();
    const uint32_t st = (uint32_t)(uintptr_t)stage + (k & 1) * 8192;
    const uint64_t rowp = (uint64_t)(uintptr_t)row;
#pragma unroll
    for (int jr = 0; jr < 8; ++jr) {
        const int r = 8 * k + jr;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rowp, r);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(rowp >> 32), r);
        const char* base = reinterpret_cast<const char*>(((uint64_t)hi << 32) | lo);
        stat_dma16(base + 16 * ((lane + jr) & 63), st + jr * 1024);
    }
}

// a[0..31] <- the fragments of the 32 rows whose base addresses lanes 0..31
// hold in `row` (lane j + 32 holds the same row as lane j), through this
// wave's 16 KiB of LDS at `stage`, given that rounds 0 and 1 were issued
// (stat_issue_round) and no other vector-memory operation of the wave is
// younger than them.  Four rounds of 8 rows, two buffers: round k+2 flies
// while round k's fragments are read.  Leaves no DMA in flight and every
// LDS read done.  K = 512.
__device__ __forceinline__ void stat_finish_rows512(frag8_t (&a)[32], const uint16_t* row, char* stage) {
    const int lane = stat_lane();
    const int j = lane & 31, half = lane >> 5, jr = j & 7;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < 3)
            __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8): round k landed, round k+1 may fly
        else
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        // chunk c = 2 ks + half of staged row jr sits at slot (c - jr) mod 64
        const char* rb = stage + (k & 1) * 8192 + jr * 1024;
        if ((j >> 3) == k) {
#pragma unroll
            for (int ks = 0; ks < 32; ++ks)
                a[ks] = *reinterpret_cast<const frag8_t*>(rb + 16 * ((2 * ks + half - jr) & 63));
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): buffer k & 1 may be overwritten
        if (k + 2 < 4) stat_issue_round(row, stage, k + 2);
    }
}

// Both steps at once (nothing to overlap with in between).
__device__ __forceinline__ void stat_load_rows512(frag8_t (&a)[32], const uint16_t* row, char* stage) {
    stat_issue_round(row, stage, 0);
    stat_issue_round(row, stage, 1);
    stat_finish_rows512(a, row, stage);
}

}  // namespace avr
