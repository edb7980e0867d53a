// msv_coop.hip -- the cooperative plan: ONE sequence per workgroup, its DP row spread over the W waves
// of the workgroup (one per SIMD of a CU), for batches of fewer sequences than the chip has CUs -- the
// shape of the reference's own benchmark programs, which score one sequence per call
// (algorithms/benchmark_helper.hpp:19-38, benchmark_MSV_1400.cpp:8-13: 1400.hmm x 3 x 3500 residues).
//
// With one sequence per wave (the latency plan) a 1400-state row is ~100 VALU issued by ONE wave,
// latency-bound at ~0.24 us per row.  Here each of the W waves owns a contiguous quarter of the row
// (64 lanes x S states) and issues ~1/W of the instructions.  The only cross-wave dependencies of a
// row t are (MSV_HMM.cpp:100-111):
//   * the j-1 neighbour of a wave's first state (the previous wave's last state at row t-1), and
//   * B(t-1) = max(N, J) + move, J being the max over ALL states.
// Neither is exchanged per row:
//   * HALO: wave w's lanes also cover the K >= 16 states just below its own (the last K states of wave
//     w-1, recomputed redundantly).  At the start of a 16-row block the halo lanes are loaded with
//     wave w-1's exact values; the halo's first state has no left neighbour (-inf), so after r rows of
//     the block only its first r+1 states can be wrong -- and wrong values are LOWER bounds (a max with
//     -inf instead of the true neighbour), which leave every max (E, J) exact.  With K >= 16 the wave's
//     own states stay exact for the whole block.
//   * SPECULATION: B = N + move, exact while every J partial stays below N (the common case off
//     homologous segments); every row ORs (J >= N) into a flag.  At the block's end the W waves
//     exchange flags and halos with ONE barrier; a flagged block is rolled back to its saved start and
//     re-run with the exact per-row B (a barrier per row to max the waves' J).
// The last partial block of a sequence (L mod 16 rows) runs that exact way too.  Bit-exact for every
// input: the same IEEE ops in the same order per state as the batch kernel (msv_kernel_body.inc).
#include "msv_kernel_impl.h"

namespace msvk {

// SA < S: the SPLIT form for tables larger than LDS (up to 2480 states): each lane's first SA states
// have their 21 residue rows in LDS, its last SB = S - SA (2 or 4) come from a lane-contiguous global table
// (L2-resident) requested four rows ahead -- the residues of a 16-row block are known at its start.
template <int W, int S, int SA = S>
__global__ __launch_bounds__(W * 64) void msv_coop_kernel(const KernelArgs a) {
#define COOP_BLOCK blockIdx.x
#define COOP_BLOCKS gridDim.x
#include "msv_coop_body.inc"
#undef COOP_BLOCK
#undef COOP_BLOCKS
}

// Several profiles' small batches in ONE launch (msv_score_grid of a few sequences, the reference's
// benchmark_MSV.cpp:32-41 shape): workgroups [p * per_profile, (p + 1) * per_profile) score profile p with
// g.p[p] -- its table in this variant's layout -- exactly as msv_coop_kernel would with a grid of
// per_profile workgroups.
template <int W, int S, int SA = S>
__global__ __launch_bounds__(W * 64) void msv_coop_grid_kernel(const GridArgs g) {
    const uint32_t profile = blockIdx.x / g.per_profile;
    const uint32_t per_profile = g.per_profile;
    const uint32_t block_in_profile = blockIdx.x - profile * per_profile;
    const KernelArgs a = g.p[profile];
#define COOP_BLOCK block_in_profile
#define COOP_BLOCKS per_profile
#include "msv_coop_body.inc"
#undef COOP_BLOCK
#undef COOP_BLOCKS
}

#define MSV_COOP_VARIANT(W_, S_)                                                                            \
    CoopVariant{W_, S_, (16 + S_ - 1) / S_ * S_, reinterpret_cast<const void*>(&msv_coop_kernel<W_, S_>), \
                "msv_coop_w" #W_ "_s" #S_, S_, reinterpret_cast<const void*>(&msv_coop_grid_kernel<W_, S_>)}
#define MSV_COOP_SPLIT_VARIANT(W_, S_, SA_)                                                                  \
    CoopVariant{W_, S_, (16 + S_ - 1) / S_ * S_, reinterpret_cast<const void*>(&msv_coop_kernel<W_, S_, SA_>), \
                "msv_coop_w" #W_ "_s" #S_ "_a" #SA_, SA_,                                                     \
                reinterpret_cast<const void*>(&msv_coop_grid_kernel<W_, S_, SA_>)}

// 448 / 960 / 1464 states with the whole table in LDS; 1984 / 2480 with the split table.
static const CoopVariant kCoop[] = {MSV_COOP_VARIANT(4, 2), MSV_COOP_VARIANT(4, 4), MSV_COOP_VARIANT(4, 6),
                                    MSV_COOP_SPLIT_VARIANT(4, 8, 6), MSV_COOP_SPLIT_VARIANT(4, 10, 6)};

const CoopVariant* coop_variants(int* count) {
    *count = static_cast<int>(sizeof(kCoop) / sizeof(kCoop[0]));
    return kCoop;
}

}  // namespace msvk
