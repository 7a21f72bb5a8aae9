// Phase probes for timing experiments (tools/probe_phases.py).  Compiled
// in only with -DAVR_PHASE_PROBES, which `make probe` sets for a separate
// library (tools/_lib/libavr_probe.so) that the tools load; the shipped
// libavr_hip.so has none of this.  A probed kernel records per wave, in a
// buffer the tool hands over, sixteen 64-bit words:
//   [0] s_memrealtime at the start (100 MHz, chip-wide)
//   [1] s_memtime at the start (shader clock)
//   [2] s_memtime when the prologue is done
//   [3] s_memtime at the end
//   [4..6] shader clocks accumulated in three phases the kernel names
//   [7] s_memrealtime at the end
//   [8..15] s_memtime marks the kernel names (AVR_PROBE_MARK(8..15))
#pragma once

// shape-selection switches of the probe tools (AVR_*_PROBE variables), read
// only by the probe and shape-probe builds (`make probe`, `make shapes`); the
// shipped library reads no such variable (tests/test_lib_abi.py)
#if defined(AVR_PHASE_PROBES) || defined(AVR_SHAPE_PROBES)
#define AVR_PROBE_ENV(name) getenv(name)
#else
#define AVR_PROBE_ENV(name) ((const char*)nullptr)
#endif

#ifdef AVR_PHASE_PROBES
#define AVR_PROBE_TU(setter)                                                                  \
    namespace {                                                                              \
    __device__ unsigned long long* avr_probe_buf = nullptr;                                   \
    __device__ int avr_probe_skip = 0;                                                        \
    }                                                                                        \
    extern "C" int setter(void* p) {                                                         \
        return hipMemcpyToSymbol(HIP_SYMBOL(avr_probe_buf), &p, sizeof(p)) == hipSuccess ? 0 : 1; \
    }                                                                                        \
    extern "C" int setter##_skip(int v) {                                                    \
        return hipMemcpyToSymbol(HIP_SYMBOL(avr_probe_skip), &v, sizeof(v)) == hipSuccess ? 0 : 1; \
    }
// phase-skip experiments (results WRONG; probe build only): a kernel skips
// the phases whose bits the tool sets, to price them
#define AVR_PROBE_SKIP(bit) (avr_probe_skip & (bit))
#define AVR_PROBE_DECL                                                  \
    unsigned long long probe_w[16] = {};                                \
    probe_w[0] = __builtin_amdgcn_s_memrealtime();                      \
    probe_w[1] = __builtin_amdgcn_s_memtime()
#define AVR_PROBE_MARK(k) probe_w[k] = __builtin_amdgcn_s_memtime()
#define AVR_PROBE_BEGIN(name) const unsigned long long probe_##name = __builtin_amdgcn_s_memtime()
#define AVR_PROBE_END(name, k) probe_w[k] += __builtin_amdgcn_s_memtime() - probe_##name
#define AVR_PROBE_COUNT(v)
#define AVR_PROBE_FLUSH(slot)                                                  \
    do {                                                                       \
        probe_w[3] = __builtin_amdgcn_s_memtime();                             \
        probe_w[7] = __builtin_amdgcn_s_memrealtime();                         \
        if (avr_probe_buf && (threadIdx.x & 63) == 0) {                        \
            _Pragma("unroll") for (int k_ = 0; k_ < 16; ++k_)                  \
                avr_probe_buf[(size_t)(slot) * 16 + k_] = probe_w[k_];          \
        }                                                                      \
    } while (0)
#else
#define AVR_PROBE_SKIP(bit) false
#define AVR_PROBE_TU(setter)
#define AVR_PROBE_DECL
#define AVR_PROBE_MARK(k)
#define AVR_PROBE_BEGIN(name)
#define AVR_PROBE_END(name, k)
#define AVR_PROBE_COUNT(v)
#define AVR_PROBE_FLUSH(slot)
#endif
