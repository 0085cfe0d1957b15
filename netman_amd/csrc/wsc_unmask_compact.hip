// wsc_unmask_compact.hip -- COMPACT (arena) instantiations of k_unmask (see wsc_unmask.inl): 4 KiB
// windows, nt loads and default-policy stores (NT = 1, profiles/r04_compact_store_policy.log); with
// and without the UTF-8 window fold (U8).
#include "wsc_unmask.inl"

namespace wsc {
template __global__ void k_unmask<true, 4, 1>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<true, 4, 1, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
}  // namespace wsc
