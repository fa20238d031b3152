// sift_gauss_ring.h -- device helpers shared by the multi-level Gaussian kernels that push their
// vertical passes into register rings (k_gauss_duo, sift_gauss_duo.hip; k_gauss_trio,
// sift_gauss_trio.hip): packed fma, wave-uniform pointers, counted vmcnt waits, the XCD-aware
// workgroup order.
#pragma once
#include <cstdint>
#include <utility>

#include <hip/hip_runtime.h>

namespace sgk {
namespace gring {

typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v pkf(f2v a, float k, f2v c) {
    return __builtin_elementwise_fma(a, f2v{k, k}, c);
}
__device__ __forceinline__ int clampd(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <int... I, class F>
__device__ __forceinline__ void unroll_seq(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}

// a wave-uniform pointer as one (the asm's "s" operand needs an SGPR pair)
__device__ __forceinline__ const char* uniform_ptr(const void* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return reinterpret_cast<const char*>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// workgroup order: blocks dealt round-robin over the 8 XCDs (observed, speed only), so logical
// block xcd * q + k runs on XCD xcd and neighbouring strips share one L2 (as k_gauss_lean)
__device__ __forceinline__ int ring_block(int bid, int nb) {
    const int q = nb / 8, r = nb % 8, xcd = bid % 8, k = bid / 8;
    return xcd < r ? xcd * (q + 1) + k : r * (q + 1) + (xcd - r) * q + k;
}

// p / 255 correctly rounded on a pair (u8_to_unit of sift_kernels.hip, packed: the same three
// IEEE operations per element)
__device__ __forceinline__ f2v u8_pair_to_unit(uint32_t a, uint32_t b) {
    const float c = 1.0f / 255.0f;
    const f2v x{(float)a, (float)b};
    const f2v q = x * f2v{c, c};
    const f2v r = __builtin_elementwise_fma(-q, f2v{255.0f, 255.0f}, x);
    return __builtin_elementwise_fma(r, f2v{c, c}, q);
}

// s_waitcnt with vmcnt = n (0 .. 63), expcnt and lgkmcnt not waited for
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt field");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void wait_lgkm0() {
    __builtin_amdgcn_s_waitcnt((15) | (3 << 14) | (7 << 4) | (0 << 8));   // lgkmcnt(0) only
}

// 5 global_load_lds_dword of one input row pair into an LDS slot (64 floats apart), lane offsets
// off[q] (bytes) from the uniform row base.  Inline asm, not __builtin_amdgcn_global_load_lds:
// the compiler's wait insertion treats every later LDS read as possibly aliasing a pending
// LDS-DMA and puts an s_waitcnt vmcnt(0) before it, which would drain the DMA ring every step;
// hidden from the compiler, the DMAs are waited for by the kernels' counted waits only.  M0 holds
// the LDS address (nothing else in these kernels uses M0).
// (the asm names M0 as clobbered: clang warns that M0 is reserved)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma_pair5(const char* base, uint32_t lds, const uint32_t (&off)[5],
                                          uint32_t ro) {
    asm volatile(
        "s_mov_b32 m0, %[l]\n\ts_nop 0\n\t"
        "global_load_lds_dword %[o0], %[b]\n\t"
        "s_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
        "global_load_lds_dword %[o1], %[b]\n\t"
        "s_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
        "global_load_lds_dword %[o2], %[b]\n\t"
        "s_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
        "global_load_lds_dword %[o3], %[b]\n\t"
        "s_add_u32 m0, m0, 0x100\n\ts_nop 0\n\t"
        "global_load_lds_dword %[o4], %[b]"
        :
        : [l] "s"(lds), [b] "s"(base), [o0] "v"(off[0] + ro), [o1] "v"(off[1] + ro),
          [o2] "v"(off[2] + ro), [o3] "v"(off[3] + ro), [o4] "v"(off[4] + ro)
        : "memory", "m0", "scc");
}
// One row pair as two global_load_lds_dwordx4 (16 B per lane, 1 KB per instruction, lane-linear
// in LDS): lanes' byte offsets off0 / off1 from the uniform base; with `masked` the second
// instruction runs on lanes 0 .. n1 - 1 only (1 <= n1: it is always issued, for the counted
// waits).
__device__ __forceinline__ void dma_pair_x4(const char* base, uint32_t lds, uint32_t off0,
                                            uint32_t off1, bool masked, int lane, int n1) {
    asm volatile(
        "s_mov_b32 m0, %[l]\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %[o0], %[b]"
        :
        : [l] "s"(lds), [b] "s"(base), [o0] "v"(off0)
        : "memory", "m0");
    if (!masked || lane < n1) {
        asm volatile(
            "s_mov_b32 m0, %[l]\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %[o1], %[b]"
            :
            : [l] "s"(lds + 1024u), [b] "s"(base), [o1] "v"(off1)
            : "memory", "m0");
    }
}
#pragma clang diagnostic pop

}  // namespace gring
}  // namespace sgk
