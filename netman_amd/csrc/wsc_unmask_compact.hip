// wsc_unmask_compact.hip -- COMPACT (arena) instantiations of k_unmask (see wsc_unmask.inl);
// each with and without the UTF-8 window fold (U8).
#include "wsc_unmask.inl"

namespace wsc {
template __global__ void k_unmask<true, 4, 0>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 4, 0, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 4, 1>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 4, 1, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 4, 2>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 4, 2, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 4, 3>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 4, 3, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 8, 0>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 8, 0, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 8, 1>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 8, 1, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 8, 2>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 8, 2, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 8, 3>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 8, 3, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
}  // namespace wsc
