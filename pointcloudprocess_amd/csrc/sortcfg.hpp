// rocPRIM onesweep configuration for the (u32 cell key, 16-byte record) sorts of the fp32
// ICP index build (grid.hip) and of the ICP query set (icp.hip).  PCP_SORT_BITS = 0 keeps
// rocPRIM's tuned gfx950 default (8 key bits per pass: 4 passes for the ~30-bit cell keys);
// 10 or 11 sorts the same keys in 3 passes.
#pragma once
#include <rocprim/device/device_radix_sort.hpp>

#ifndef PCP_SORT_BITS
#define PCP_SORT_BITS 0
#endif

namespace pcp {
#if PCP_SORT_BITS
using RecSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 6>, rocprim::kernel_config<1024, 6>,
                                        PCP_SORT_BITS, rocprim::block_radix_rank_algorithm::match>>;
#else
using RecSortConfig = rocprim::default_config;
#endif
}  // namespace pcp
