// wsc_u8.hpp -- UTF-8 (Go utf8.Valid, websocket_frame.go:71-73, websocket.go:170-172) as DFA
// transition maps, shared by the chip-wide check (k_u8_check, wsc_kernels.hip) and the unmask,
// which folds the text windows it has just unmasked (k_unmask, wsc_unmask.inl).
//
// The DFA has 9 states, 0 = between characters, 8 = reject.  What a run of bytes does to it is a
// map from entry state to exit state.  A map is 8 bytes: byte s = the state after the bytes when
// entering in state s (0..7), 0xFF = reject; the reject state itself is absorbing and not stored.
// With this encoding a map is a v_perm_b32 table: applying map b after map a is two v_perm_b32
// (a's bytes select from b; 0xFF selects 0xFF), and one input byte is one 8-byte table row.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wsc {

__device__ __forceinline__ uint32_t u8_step(uint32_t s, uint32_t b) {
    switch (s) {
    case 0:
        if (b < 0x80) return 0;
        if (b >= 0xC2 && b <= 0xDF) return 1;
        if (b == 0xE0) return 4;
        if (b == 0xED) return 5;
        if (b >= 0xE1 && b <= 0xEF) return 2;
        if (b == 0xF0) return 6;
        if (b >= 0xF1 && b <= 0xF3) return 3;
        if (b == 0xF4) return 7;
        return 8;
    case 1: return (b >= 0x80 && b <= 0xBF) ? 0 : 8;
    case 2: return (b >= 0x80 && b <= 0xBF) ? 1 : 8;
    case 3: return (b >= 0x80 && b <= 0xBF) ? 2 : 8;
    case 4: return (b >= 0xA0 && b <= 0xBF) ? 1 : 8;
    case 5: return (b >= 0x80 && b <= 0x9F) ? 1 : 8;
    case 6: return (b >= 0x90 && b <= 0xBF) ? 2 : 8;
    case 7: return (b >= 0x80 && b <= 0x8F) ? 2 : 8;
    default: return 8;
    }
}

__device__ __forceinline__ uint64_t u8m_id() { return 0x0706050403020100ull; }
__device__ __forceinline__ uint64_t u8m_ascii() { return 0xFFFFFFFFFFFFFF00ull; }   // 0 -> 0, mid-character -> reject
__device__ __forceinline__ uint64_t u8m_then(uint64_t a, uint64_t b) {   // a, then b
    const uint32_t bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_perm(bh, bl, (uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_perm(bh, bl, (uint32_t)(a >> 32));
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ uint32_t u8m_get(uint64_t m, uint32_t st) {   // st: 0..7, or >= 8 = reject
    return st > 7 ? 0xFFu : (uint32_t)(m >> (8 * st)) & 0xFFu;
}

// LDS tables of one workgroup: tab[byte] = the map of that single byte; tab8[state][byte] = the
// next state (8 = reject); stage = one 4 KiB restage buffer per wave (64 chunks padded to 80 B).
struct U8Lds {
    uint64_t tab[256];
    uint8_t tab8[9 * 256];
};
constexpr uint32_t U8_STAGE = 64 * 5;   // uint4 per wave
// every thread of a 256-thread workgroup fills its byte's entries (caller syncs)
__device__ __forceinline__ void u8_tables_init(U8Lds& t, uint32_t byte) {
    uint64_t m = 0;
    for (uint32_t st = 0; st < 8; ++st) {
        const uint32_t ns = u8_step(st, byte);
        m |= (uint64_t)(ns == 8 ? 0xFFu : ns) << (8 * st);
        t.tab8[st * 256 + byte] = (uint8_t)ns;
    }
    t.tab8[8 * 256 + byte] = 8;
    t.tab[byte] = m;
}

// one level of the in-row composition: lanes that are multiples of 2*DD take "own map, then the map
// of lane + DD" (DPP row_shl:DD -- lane i reads lane i + DD of its 16-lane row)
template <int DD>
__device__ __forceinline__ void u8m_row_level(uint32_t& mlo, uint32_t& mhi, uint32_t lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mlo, 0x100 | DD, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mhi, 0x100 | DD, 0xF, 0xF, false);
    if ((lane & (2 * DD - 1)) == 0) {
        const uint64_t c = u8m_then((uint64_t)mhi << 32 | mlo, (uint64_t)hi << 32 | lo);
        mlo = (uint32_t)c;
        mhi = (uint32_t)(c >> 32);
    }
}
// The 16-lane rows' maps in lane order (DPP row shifts), left in lanes 0, 16, 32, 48.
__device__ __forceinline__ uint64_t u8_row_maps(uint64_t pm, uint32_t lane) {
    uint32_t mlo = (uint32_t)pm, mhi = (uint32_t)(pm >> 32);
    u8m_row_level<1>(mlo, mhi, lane);
    u8m_row_level<2>(mlo, mhi, lane);
    u8m_row_level<4>(mlo, mhi, lane);
    u8m_row_level<8>(mlo, mhi, lane);
    return (uint64_t)mhi << 32 | mlo;
}
// The map of a 4 KiB wave step (the 64 lanes' chunk maps in lane order), wave-uniform.
__device__ __forceinline__ uint64_t u8_wave_map(uint64_t pm, bool plain, uint32_t lane) {
    if (__ballot(!plain) == 0)            // ASCII (or empty) everywhere: one constant map
        return __ballot(pm == u8m_ascii()) ? u8m_ascii() : u8m_id();
    const uint64_t rm = u8_row_maps(pm, lane);
    const uint32_t mlo = (uint32_t)rm, mhi = (uint32_t)(rm >> 32);
    uint64_t m = u8m_id();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        // readlane returns int: widen through uint32_t (no sign extension into the high word)
        const uint32_t rlo = (uint32_t)__builtin_amdgcn_readlane(mlo, 16 * r);
        const uint32_t rhi = (uint32_t)__builtin_amdgcn_readlane(mhi, 16 * r);
        m = u8m_then(m, (uint64_t)rhi << 32 | rlo);
    }
    return m;
}

// Coalesced 16 B-per-lane pieces (piece k at 1024 k + 16 lane of a 4 KiB step) restaged through the
// wave's LDS buffer into one contiguous 64-byte chunk per lane (chunks padded to 80 B: the 16 lanes
// of a ds_read_b128 phase then hit 16 distinct bank groups).
template <typename V>
__device__ __forceinline__ void u8_restage(uint4* sw, V (&q)[4], uint32_t lane) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t b = 1024u * k + 16u * lane;
        sw[(b >> 6) * 5 + ((b >> 4) & 3)] = make_uint4(q[k][0], q[k][1], q[k][2], q[k][3]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 t = sw[lane * 5 + k];
        q[k][0] = t.x; q[k][1] = t.y; q[k][2] = t.z; q[k][3] = t.w;
    }
    __builtin_amdgcn_wave_barrier();
}

// The map of one lane's 64-byte chunk (nk valid bytes, each dword XORed with `mask`); plain = no
// non-ASCII byte among them.  Inside a chunk the first 4 bytes compose full maps (two v_perm per
// byte from the 8-byte rows of `tab`); every entry state that survives them is then in one state
// X, which steps through the other 60 bytes one byte-table read each (`tab8[X][byte]`, state 8 =
// reject, absorbing): two VALU ops and one LDS read per byte.
// How a wave folds chunks that end early (the last of an item):
enum U8Part : uint32_t {
    U8P_LANE = 0,   // the partial chunk's lane alone folds it byte by byte with full maps
    U8P_WAVE = 1,   // the whole wave takes the chain steps predicated on each byte being valid
    U8P_NONE = 2,   // the caller's chunks are always whole (the unmask's window fold)
};
template <uint32_t NCH, U8Part PART, typename V>
__device__ __forceinline__ uint64_t u8_chunk_map(const U8Lds& t, const V (&v)[4], uint32_t mask, uint32_t nk,
                                                 bool& plain) {
    // byte i of the chunk, unmasked (i constant after unrolling)
    auto dw = [&](uint32_t j) -> uint32_t { return (uint32_t)v[j >> 2][j & 3] ^ mask; };
    uint32_t hib = 0;
    if (nk >= 64) {
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) hib |= dw(j);
        hib &= 0x80808080u;
    } else {
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) {
            const uint32_t lim = nk > 4u * j ? (nk - 4u * j >= 4 ? 4u : nk - 4u * j) : 0u;
            const uint32_t keep = lim >= 4 ? 0xFFFFFFFFu : ((1u << (8 * lim)) - 1u);
            hib |= dw(j) & keep & 0x80808080u;
        }
    }
    plain = nk == 0 || hib == 0;
    // nothing to fold / ASCII only (a function: not kept live across the fold)
    auto trivial = [nk]() -> uint64_t { return nk == 0 ? u8m_id() : u8m_ascii(); };
    if (PART == U8P_LANE && plain) return trivial();
    if (__ballot(!plain) == 0) return trivial();
    if (PART == U8P_LANE && nk < 64) {
        // (unrolled with a guard: a dynamic index into the chunk would go to scratch)
        uint32_t lo = 0x03020100u, hi = 0x07060504u;
#pragma unroll
        for (uint32_t i = 0; i < 64; ++i) {
            if (i < nk) {
                const uint64_t e = t.tab[(dw(i >> 2) >> (8 * (i & 3))) & 0xFFu];
                const uint32_t tl = (uint32_t)e, th = (uint32_t)(e >> 32);
                lo = (uint32_t)__builtin_amdgcn_perm(th, tl, lo);
                hi = (uint32_t)__builtin_amdgcn_perm(th, tl, hi);
            }
        }
        return (uint64_t)hi << 32 | lo;
    }
    // Every entry state that survives the first 4 bytes is in ONE state X there: a survivor
    // must be in state 0 just before the first lead byte (a lead in a non-zero state rejects),
    // and 4 continuation bytes reject every state (at most 3 are owed).  So the first 4 bytes
    // compose full maps, the others step the single state X, and the chunk's map is the
    // prefix map with every surviving entry sent to the final state.  NCH independent chains of
    // 64 / NCH bytes, interleaved byte by byte (latency: each chain is a dependent sequence of
    // LDS reads), are composed in order at the end.
    // A partial chunk's map must leave a character that the item ends inside owed, not rejected
    // by padding.  U8P_LANE: that lane folded it above, byte by byte, and the wave runs both
    // forms.  U8P_WAVE: the wave folds all its chunks one way -- the chain steps predicated on
    // the byte being valid as soon as one chunk is partial, a chain with at most 4 valid bytes
    // keeping its full-map composition (cheaper where few waves hold a partial chunk: 64 KiB
    // items; dearer where most do: 1 KiB items).
    const bool part = PART == U8P_WAVE && __ballot(!plain && nk < 64) != 0;
    constexpr uint32_t CW = 16 / NCH, CB = 4 * CW;   // dwords / bytes per chain
    uint32_t clo[NCH], chi[NCH], st[NCH];
#pragma unroll
    for (uint32_t c = 0; c < NCH; ++c) {
        const uint32_t d0 = dw(c * CW);
        uint32_t l = 0x03020100u, h = 0x07060504u;
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            const uint64_t e = t.tab[(d0 >> (8 * i)) & 0xFFu];
            const uint32_t tl = (uint32_t)e, th = (uint32_t)(e >> 32);
            const uint32_t l2 = (uint32_t)__builtin_amdgcn_perm(th, tl, l);
            const uint32_t h2 = (uint32_t)__builtin_amdgcn_perm(th, tl, h);
            const bool take = !part || c * CB + i < nk;
            l = take ? l2 : l;
            h = take ? h2 : h;
        }
        uint32_t x = l & h;             // non-rejected bytes all equal X, rejects are 0xFF
        x &= x >> 16;
        x &= x >> 8;
        x &= 0xFFu;
        st[c] = x > 7 ? 8u : x;
        clo[c] = l;
        chi[c] = h;
    }
    // one v_perm per byte builds the table index st << 8 | byte (and, depending on st, keeps
    // the compiler from hoisting the byte extractions into live registers)
#pragma unroll
    for (uint32_t j = 1; j < CW; ++j) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
#pragma unroll
            for (uint32_t c = 0; c < NCH; ++c) {
                const uint32_t ns = t.tab8[__builtin_amdgcn_perm(st[c], dw(c * CW + j), i | 4u << 8 | 0x0Cu << 16 | 0x0Cu << 24)];
                st[c] = (!part || c * CB + 4 * j + i < nk) ? ns : st[c];
            }
        }
    }
    uint64_t m = u8m_id();
#pragma unroll
    for (uint32_t c = 0; c < NCH; ++c) {
        const uint32_t fr = (st[c] > 7 ? 0xFFu : st[c]) * 0x01010101u;
        uint32_t l = (uint32_t)__builtin_amdgcn_perm(fr, fr, clo[c]);   // 0..7 -> final state
        uint32_t h = (uint32_t)__builtin_amdgcn_perm(fr, fr, chi[c]);
        if (part && nk <= c * CB + 4) {   // (at most 4 bytes: the composed map itself)
            l = clo[c];
            h = chi[c];
        }
        m = c == 0 ? ((uint64_t)h << 32 | l) : u8m_then(m, (uint64_t)h << 32 | l);
    }
    return plain ? trivial() : m;
}

}  // namespace wsc
