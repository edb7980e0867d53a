// vit_kernel.h -- device-side interface of the Viterbi stage, shared by vit_kernel.hip and
// the C-ABI layer (vit_device.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace vitk {

constexpr int kRows = 20;        // residue rows of the score tables (codes >= 20 are flagged, not scored)
constexpr int kTransitions = 7;  // per-slot transition arrays, see VitArgs::ttab
constexpr int kLanes = 64;       // one sequence per wave: 64 lanes own the DP row
constexpr int kLdsLimit = 163840;

// Slot arrays of the transition table, per lane slot q (state k = lane * S + q + 1):
//   MM_IN, IM_IN, DM_IN : into M_k from node k-1;   MI, II : out of node k into I_k;
//   MD_IN, DD_IN        : into D_k from node k-1.
// -inf where the transition does not exist (node 0, I at node LENG, padding slots beyond LENG).
enum : int { MM_IN = 0, IM_IN = 1, DM_IN = 2, MI = 3, II = 4, MD_IN = 5, DD_IN = 6 };

struct VitArgs {
    const float2* etab;         // match scores  [20][S/2][64] float2 (padding slots -inf)
    const float2* itab;         // insert scores [20][S/2][64] float2 (ISC variants only)
    const float2* ttab;         // transitions   [7][S/2][64] float2
    const uint8_t* residues;    // CSR residue codes
    const uint64_t* offsets;    // n + 1
    const uint32_t* select;     // optional: the sequence indices to score (else 0 .. n-1)
    const uint32_t* select_count;  // optional device count of `select` entries (else n)
    const float2* lentab;       // [lentab_n] {tr_loop, tr_move} by length (host logf)
    float* scores;              // written at the sequence index
    uint32_t* counter;          // {dequeue head, leavers: workgroups (vit_kernel) / waves (team)}: zero on entry and exit
    uint32_t* errors;           // sticky error bits (msvk::kErrBadResidue / kErrTooLong)
    uint64_t n;
    uint32_t lentab_n;
    float tr_B_Mk, tr_E_C, tr_E_J;
    // diagnostic timeline (tools/vit_timeline.py; nullptr in production, team kernels only): per list entry j
    // {realtime start, end, hw id << 32 | wave, length}, then per wave {entry, tables staged, exit, XCC id}
    uint64_t* stamps;
};

// One compiled instantiation: S states per lane (G = 64 lanes per sequence, covers 64 * S states), the first
// `ntreg` transition arrays in VGPRs and the rest in LDS, match scores in LDS (elds) or read from L2 every
// row, informative insert scores (isc, read from L2) or HMMER3's zero insert scores; `waves` 64-lane waves
// per workgroup.  `pick`: the automatic choice for its S (one per S and insert mode, chosen by measurement,
// profiles/r04_vit_tune_*.jsonl); the others are A/B candidates reachable through msv_vit_profile_set_variant.
//
// team > 1 (vit_team.hip, round 5): one sequence per TEAM of `team` waves (virtual lane v = w * 64 + lane
// holds states v * S + 1 .. v * S + S; the tables' lane axis is the team's 64 * team virtual lanes), with
// waves / team teams per workgroup.
struct VitVariant {
    int S;
    int ntreg;
    bool elds, isc;
    int waves;  // per workgroup
    bool pick;
    const void* fn;
    const char* name;
    int lds_bytes;
    int team = 1;  // waves per sequence
    int states() const { return kLanes * S * team; }
    int chunks() const { return (S + 1) / 2; }      // float2 chunks per lane in the table layouts
    int sequences_per_block() const { return waves / team; }
};

const VitVariant* vit_variants(int* count);      // every variant: vit_kernel.hip's, then the team family
const VitVariant* vit_team_variants(int* count);  // vit_team.hip
hipError_t vit_launch(const VitVariant& v, uint32_t blocks, const VitArgs& args, hipStream_t stream,
                      hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
// MSV filter survivors: P-value of every MSV score (msv_pvalue_of, STATS LOCAL MSV), written to pvalues
// when non-null, and the indices with P <= threshold written to select in the order's order (a stable
// compaction: two launches), their number to *count.
hipError_t launch_select(const float* scores, const uint64_t* offsets, const uint32_t* order, uint64_t n, float mu,
                         float lambda, double threshold, double* pvalues, uint32_t* select, uint32_t* count,
                         hipStream_t stream);

}  // namespace vitk
