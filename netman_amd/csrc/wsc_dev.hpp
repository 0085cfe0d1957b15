// wsc_dev.hpp -- small gfx950 device helpers shared by the decode (wsc_kernels.hip) and encode
// (wsc_encode.hip) kernels: byte masks, unaligned 16-byte gathers, 16-byte (non-temporal) access.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wsc {

__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t r) {
    r &= 31;
    return r ? (x >> r) | (x << (32 - r)) : x;
}

__device__ __forceinline__ uint32_t bytes_to_mask(uint32_t lo, uint32_t hi) {
    // byte lanes [lo, hi) of a dword, lo <= hi <= 4
    const uint32_t a = lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo));
    const uint32_t b = hi >= 4 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu << (8 * hi));
    return a & b;
}

typedef unsigned int u32x4u_ld __attribute__((ext_vector_type(4), aligned(1)));

// 16 bytes starting at src + off (off may be unaligned); bytes outside [0, n) read as 0.  Inside
// the buffer this is ONE byte-aligned 16-byte load (gfx950 global memory takes unaligned
// addresses; a wave's 64 loads still cover one contiguous ~1 KiB range); at the edges, byte loads.
__device__ __forceinline__ uint4 load16_unaligned(const uint8_t* __restrict__ src, int64_t off,
                                                  uint64_t n) {
    if (off >= 0 && (uint64_t)off + 16 <= n) {
        const u32x4u_ld t = *reinterpret_cast<const u32x4u_ld*>(src + off);
        return make_uint4(t.x, t.y, t.z, t.w);
    }
    uint32_t t[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int64_t q = off + j;
        if (q >= 0 && (uint64_t)q < n) t[j >> 2] |= (uint32_t)src[q] << (8 * (j & 3));
    }
    return make_uint4(t[0], t[1], t[2], t[3]);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// load16_unaligned with the cache policy of NT bit 0 (non-temporal: a stream read once)
template <int NT>
__device__ __forceinline__ uint4 load16u(const uint8_t* __restrict__ src, int64_t off, uint64_t n) {
    if constexpr ((NT & 1) != 0) {
        if (off >= 0 && (uint64_t)off + 16 <= n) {
            const u32x4u_ld t = __builtin_nontemporal_load(reinterpret_cast<const u32x4u_ld*>(src + off));
            return make_uint4(t.x, t.y, t.z, t.w);
        }
    }
    return load16_unaligned(src, off, n);
}

template <int NT>
__device__ __forceinline__ u32x4 ld16v(const uint8_t* p) {
    if constexpr (NT & 1) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
}
template <int NT>
__device__ __forceinline__ void st16v(uint8_t* p, u32x4 v) {
    if constexpr (NT & 2) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else *reinterpret_cast<u32x4*>(p) = v;
}
// Buffer-instruction window I/O (k_unmask in place, NT >= 16): one resource per wave window,
// 32-bit lane offsets, explicit gfx950 cache-policy bits (aux bit 0 = sc0, bit 1 = nt, bit 4 =
// sc1).  tools/hbm_ceiling.hip "sweep": the same in-place XOR through buffer ops with nt loads
// and nt(+sc1) stores streams 1 GiB 9-10 % faster than through 64-bit global addresses.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t win_rsrc(uint8_t* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ u32x4 ld16b(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}
template <int AUX>
__device__ __forceinline__ void st16b(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}

// Byte-aligned stores (gfx950 global memory takes unaligned dword/dwordx2/dwordx4 addresses; the
// compiler emits the same instructions for align-1 accesses).
typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef unsigned int u32x2u __attribute__((ext_vector_type(2), aligned(1)));
typedef unsigned int u32u __attribute__((aligned(1)));
typedef unsigned short u16u __attribute__((aligned(1)));
template <int NT>
__device__ __forceinline__ void st16u(uint8_t* p, u32x4 v) {
    const u32x4u t = {v.x, v.y, v.z, v.w};
    if constexpr (NT & 2) __builtin_nontemporal_store(t, reinterpret_cast<u32x4u*>(p));
    else *reinterpret_cast<u32x4u*>(p) = t;
}

// bytes [sh, sh + 16) of the 16-byte vector x followed by zeros (sh in [0, 16))
__device__ __forceinline__ u32x4 shr_bytes16(u32x4 x, uint32_t sh) {
    const uint32_t d[8] = {x.x, x.y, x.z, x.w, 0u, 0u, 0u, 0u};
    const uint32_t q = sh >> 2, rb = sh & 3;
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t lo = d[j], hi = d[j + 1];
        if (q == 1) { lo = d[j + 1]; hi = d[j + 2]; }
        else if (q == 2) { lo = d[j + 2]; hi = d[j + 3]; }
        else if (q == 3) { lo = d[j + 3]; hi = d[j + 4]; }
        o[j] = __builtin_amdgcn_alignbyte(hi, lo, rb);
    }
    return o;
}

// bytes [g, g + 16) of the 32 bytes x then y, g in [0, 16]: two select levels and an alignbyte per
// dword (named values, not an array: selects between array elements became a dynamically indexed
// private array, which the compiler promoted to LDS)
__device__ __forceinline__ u32x4 funnel16(u32x4 x, u32x4 y, uint32_t g) {
    const bool c8 = (g & 8) != 0, c4 = (g & 4) != 0;
    const uint32_t e0 = c8 ? x.z : x.x, e1 = c8 ? x.w : x.y, e2 = c8 ? y.x : x.z;
    const uint32_t e3 = c8 ? y.y : x.w, e4 = c8 ? y.z : y.x, e5 = c8 ? y.w : y.y;
    const uint32_t f0 = c4 ? e1 : e0, f1 = c4 ? e2 : e1, f2 = c4 ? e3 : e2, f3 = c4 ? e4 : e3, f4 = c4 ? e5 : e4;
    const uint32_t b = g & 3;
    const u32x4 o = {__builtin_amdgcn_alignbyte(f1, f0, b), __builtin_amdgcn_alignbyte(f2, f1, b),
                     __builtin_amdgcn_alignbyte(f3, f2, b), __builtin_amdgcn_alignbyte(f4, f3, b)};
    return g >= 16 ? y : o;
}

// Store bytes [lo, hi) of the 16-byte vector x at p (p = where byte lo goes; 0 <= lo < hi <= 16):
// at most four stores of 8, 4, 2 and 1 bytes (one of 16 for a whole piece); nothing else is touched.
template <int NT>
__device__ __forceinline__ void store_run(uint8_t* p, u32x4 x, uint32_t lo, uint32_t hi) {
    const uint32_t n = hi - lo;
    if (n == 16) { st16u<NT>(p, x); return; }
    u32x4 y = shr_bytes16(x, lo);
    if (n & 8) {
        *reinterpret_cast<u32x2u*>(p) = u32x2u{y.x, y.y};
        p += 8;
        y = u32x4{y.z, y.w, 0u, 0u};
    }
    if (n & 4) {
        *reinterpret_cast<u32u*>(p) = y.x;
        p += 4;
        y = u32x4{y.y, y.z, 0u, 0u};
    }
    if (n & 2) {
        *reinterpret_cast<u16u*>(p) = (uint16_t)y.x;
        p += 2;
        y.x >>= 16;
    }
    if (n & 1) *p = (uint8_t)y.x;
}

// XCD runs of blocks for the streaming kernels (unmask, encode copy).  Blocks are dealt
// round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch: blocks b and b + 8 share
// one), so with the identity map neighbouring blocks' windows sit in different XCDs' L2s.  With
// R > 1 each chunk of 8R blocks is remapped so that XCD x (b mod 8) takes R consecutive logical
// blocks while the eight XCDs still stream one 8R-block region together.  A bijection on the full
// chunks (the tail keeps the identity); placement changes speed only, never results.
__device__ __forceinline__ uint32_t xcd_run_block(uint32_t bid, uint32_t grid, uint32_t R) {
    if (R <= 1) return bid;
    const uint32_t chunk = 8u * R;
    if (bid >= grid / chunk * chunk) return bid;
    const uint32_t j = bid % chunk;
    return bid - j + (j & 7u) * R + (j >> 3);
}

template <int NT>
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    const u32x4 t = ld16v<NT>(p);
    return make_uint4(t.x, t.y, t.z, t.w);
}
template <int NT>
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) {
    u32x4 t = {v.x, v.y, v.z, v.w};
    st16v<NT>(p, t);
}

// Staged pipeline: the LAST workgroup of a grid to finish writes fin_seq to the host-visible word
// (wsc_api.cpp fin_wait) -- called by thread 0 of every workgroup after a __syncthreads, once its
// workgroup's accesses to the walk's scratch are done.  A grid is up to 2^16+ workgroups: one
// device-scope counter would serialise them (measured 5.9 ms for 64 Ki), so the count is
// two-level -- FIN_GROUPS counters a cache line apart, each finished by its last workgroup, which
// bumps the top counter.  Every level re-arms itself for the next launch.  Vector atomics only.
constexpr uint32_t FIN_GROUPS = 256, FIN_STRIDE = 32;   // fin_ctr: (FIN_GROUPS + 1) * FIN_STRIDE words
__device__ __forceinline__ void fin_signal(uint32_t* fin_ctr, uint32_t* fin_host, uint32_t fin_seq) {
    const uint32_t g = blockIdx.x % FIN_GROUPS;
    const uint32_t in_g = (gridDim.x - g + FIN_GROUPS - 1) / FIN_GROUPS;   // workgroups of group g
    uint32_t* cg = fin_ctr + (1 + g) * FIN_STRIDE;
    if (__hip_atomic_fetch_add(cg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_g - 1) {
        __hip_atomic_store(cg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t groups = gridDim.x < FIN_GROUPS ? gridDim.x : FIN_GROUPS;
        if (__hip_atomic_fetch_add(fin_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1) {
            __hip_atomic_store(fin_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            __hip_atomic_store(fin_host, fin_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __threadfence_system();
        }
    }
}

}  // namespace wsc
