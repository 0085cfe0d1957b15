// wsc_unmask_inplace.hip -- in-place instantiations of k_unmask (see wsc_unmask.inl);
// each with and without the UTF-8 window fold (U8).
#include "wsc_unmask.inl"

namespace wsc {
template __global__ void k_unmask<false, 4, 0>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 0, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 1>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 1, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 2>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 2, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 3>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 3, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 0>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 0, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 1>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 1, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 2>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 2, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 3>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 3, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
// buffer-instruction windows: nt loads, stores with aux (NT >> 4) = nt / nt sc1 / sc0 nt sc1
template __global__ void k_unmask<false, 4, 35>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 35, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 291>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 291, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 307>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 307, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 35>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 35, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 291>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 291, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 307>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 8, 307, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
}  // namespace wsc
