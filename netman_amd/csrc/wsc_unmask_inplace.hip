// wsc_unmask_inplace.hip -- in-place instantiations of k_unmask (see wsc_unmask.inl): 4 KiB windows
// through buffer instructions, nt loads and sc0 nt sc1 stores (NT = 307); with and without the UTF-8
// window fold (U8).  Other windows / cache policies were measured slower (r01_tune_*,
// r02_unmask_policy.log) and are built only by A/B variant builds (tools/build_variant.sh).
#include "wsc_unmask.inl"

namespace wsc {
template __global__ void k_unmask<false, 4, 307>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
template __global__ void k_unmask<false, 4, 307, 1, true>(uint8_t*, const uint8_t*, uint64_t, uint64_t, const Span*, const uint32_t*, const wsc_summary*, uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t, U8Win);
}  // namespace wsc
