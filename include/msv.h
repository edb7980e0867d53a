/*
 * msv.h -- C-ABI of the MI355X-native MSV (Multiple Segment Viterbi) scoring engine.
 *
 * This is the drop-in boundary for the reference's single hot path, the class
 * MSV_HMM (algorithms/MSV_HMM.hpp:17-44 of IvanTyulyandin/HMM_FASTA_Viterbi).  Plain C types
 * only: no HIP, no torch, no C++ in the signatures.  Every entry point cites the reference
 * interface it replaces.  All functions return an msv_status; nothing prints and continues
 * (the reference's check_errors prints and continues, MSV_HMM.cpp:198-203).
 *
 * Ownership: the caller owns every buffer it passes; the library owns the device buffers held
 * by an msv_profile.  One msv_profile may be used by one host thread at a time (the reference
 * MSV_HMM is likewise not thread-safe, MSV_HMM.hpp:33-34); separate profiles are independent.
 * From that one thread, a profile's device launches may go to any streams: every launch takes
 * its own dequeue counter (one of 8 slots, reused only after the slot's previous launch), so
 * launches of one profile on different streams may overlap.
 *
 * Residues cross the boundary as codes 0..19 in the reference's alphabetical order
 * A C D E F G H I K L M N P Q R S T V W Y (MSV_HMM.cpp:29-31), without the '#' sentinel that
 * the reference prepends (FASTA_protein_sequences.cpp:19-20), in a CSR layout:
 * sequence s is residues[offsets[s] .. offsets[s+1]).
 */
#ifndef MSV_H_
#define MSV_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum msv_status {
    MSV_OK = 0,
    MSV_ERR_INVALID_ARGUMENT = 1, /* null pointer, bad size, bad offsets                       */
    MSV_ERR_IO = 2,               /* file cannot be opened (reference: "Failed to open", Profile_HMM.cpp:50-53) */
    MSV_ERR_PARSE = 3,            /* malformed .hmm / FASTA                                    */
    MSV_ERR_BAD_RESIDUE = 4,      /* residue code >= 20 (reference: std::out_of_range from amino_acid_num.at, MSV_HMM.cpp:101) */
    MSV_ERR_SEQUENCE_TOO_LONG = 5,/* longer than the device transition table (msv_profile_reserve_length) */
    MSV_ERR_UNSUPPORTED_MODEL = 6,/* model length outside the compiled kernel family          */
    MSV_ERR_NO_DEVICE = 7,        /* no HIP device / bad device ordinal                        */
    MSV_ERR_HIP = 8,              /* a HIP runtime call failed                                 */
    MSV_ERR_OUT_OF_MEMORY = 9,
    MSV_ERR_RCCL = 10             /* an RCCL call failed (multi-GPU context)                   */
} msv_status;

typedef struct msv_hmm msv_hmm;         /* parsed HMMER3 profile (host)            */
typedef struct msv_fasta msv_fasta;     /* parsed FASTA, residues packed as codes  */
typedef struct msv_profile msv_profile; /* device-resident MSV scoring profile     */

/* ---------------------------------------------------------------------------------------- */
/* General                                                                                   */
/* ---------------------------------------------------------------------------------------- */
const char* msv_status_string(msv_status status);
const char* msv_version(void);
msv_status msv_device_count(int* count);

/* ---------------------------------------------------------------------------------------- */
/* Host: HMMER3 profile parser -- replaces Profile_HMM::Profile_HMM (Profile_HMM.cpp:48-60)  */
/* ---------------------------------------------------------------------------------------- */
msv_status msv_hmm_read(const char* path, msv_hmm** out);
void msv_hmm_destroy(msv_hmm* hmm);
/* LENG + 1: includes the dummy node M0 (Profile_HMM.cpp:66-71) */
size_t msv_hmm_model_length(const msv_hmm* hmm);
const char* msv_hmm_name(const msv_hmm* hmm);
/* {msv_mu, msv_lambda, viterbi_mu, viterbi_lambda, forward_theta, forward_lambda} (Profile_HMM.hpp:33-43) */
void msv_hmm_stats(const msv_hmm* hmm, float out6[6]);
/* probabilities exp(-x) as parsed (Profile_HMM.cpp:35-45): [model_length][20], [model_length][20], [model_length][7] */
const float* msv_hmm_match_emissions(const msv_hmm* hmm);
const float* msv_hmm_insert_emissions(const msv_hmm* hmm);
const float* msv_hmm_transitions(const msv_hmm* hmm);

/* MSV host precompute -- replaces MSV_HMM::MSV_HMM (MSV_HMM.cpp:35-57).
 * emission_scores: caller buffer of 20 * model_length floats, residue-major,
 * emission_scores[r * model_length + k] = logf(p_k[r] / bg[r]); column 0 = -inf. */
msv_status msv_hmm_msv_scores(const msv_hmm* hmm, float* emission_scores, float* tr_B_Mk, float* tr_E_C,
                              float* tr_E_J);

/* Per-sequence transitions -- replaces MSV_HMM::init_transitions_depend_on_seq (MSV_HMM.cpp:59-64);
 * L excludes the '#' sentinel. */
void msv_sequence_transitions(uint64_t L, float* tr_loop, float* tr_move);

/* ---------------------------------------------------------------------------------------- */
/* Host: FASTA reader -- replaces FASTA_protein_sequences (FASTA_protein_sequences.cpp:9-44) */
/* Same record semantics (lines joined, records with a symbol outside the 20 amino acids     */
/* dropped, empty records kept); residues are packed straight into the CSR code stream.     */
/* A '#' inside a record is kept by the reference parser and only fails at scoring time;    */
/* here it is stored as code 255, which the scorer rejects with MSV_ERR_BAD_RESIDUE.         */
/* ---------------------------------------------------------------------------------------- */
msv_status msv_fasta_read(const char* path, msv_fasta** out);
void msv_fasta_destroy(msv_fasta* fasta);
size_t msv_fasta_count(const msv_fasta* fasta);
size_t msv_fasta_rejected(const msv_fasta* fasta);
const uint8_t* msv_fasta_codes(const msv_fasta* fasta);     /* offsets[count] bytes   */
const uint64_t* msv_fasta_offsets(const msv_fasta* fasta);  /* count + 1 entries      */
const char* msv_fasta_header(const msv_fasta* fasta, size_t i); /* header line without '>' */

/* ---- FASTA ingest on the GPU -----------------------------------------------
 * The same records as msv_fasta_read (bit-identical codes, offsets, header spans, rejected count),
 * parsed by a chain of tile-scan kernels from FASTA text resident in HBM, so a batch can go from
 * file bytes to scores without a host-side parse.  Results stay in device memory:
 *   codes   : residues() bytes, offsets: count() + 1 uint64 (the scorer's CSR input as is),
 *   spans   : 2 * count() uint64, (start, length) of each header inside the text (no '>').
 * msv_fasta_parse_device takes text already in device memory (n < 2^32 - 2^16 bytes);
 * msv_fasta_read_device reads a file through pinned 64 MiB pieces (read/copy overlapped) and keeps
 * its own device copy of the text (msv_fasta_device_text).  Synchronous w.r.t. `stream`. */
typedef struct msv_fasta_device msv_fasta_device;
msv_status msv_fasta_parse_device(int device, const uint8_t* d_text, uint64_t n, void* stream,
                                  msv_fasta_device** out);
msv_status msv_fasta_read_device(int device, const char* path, void* stream, msv_fasta_device** out);
void msv_fasta_device_destroy(msv_fasta_device* fasta);
uint64_t msv_fasta_device_count(const msv_fasta_device* fasta);
int msv_fasta_device_device(const msv_fasta_device* fasta);           /* the GPU holding it, -1 for NULL */
uint64_t msv_fasta_device_rejected(const msv_fasta_device* fasta);
uint64_t msv_fasta_device_residues(const msv_fasta_device* fasta);
uint64_t msv_fasta_device_max_length(const msv_fasta_device* fasta);  /* longest record */
const uint8_t* msv_fasta_device_codes(const msv_fasta_device* fasta);          /* device pointer */
const uint64_t* msv_fasta_device_offsets(const msv_fasta_device* fasta);       /* device pointer */
const uint64_t* msv_fasta_device_header_spans(const msv_fasta_device* fasta);  /* device pointer */
const uint8_t* msv_fasta_device_text(const msv_fasta_device* fasta);  /* device copy, or NULL */
/* Copies codes / offsets / spans to host buffers sized as above (any may be NULL). */
msv_status msv_fasta_device_download(const msv_fasta_device* fasta, uint8_t* codes, uint64_t* offsets,
                                     uint64_t* spans);

/* Letters -> codes (A..Y -> 0..19).  Any other byte -> MSV_ERR_BAD_RESIDUE. */
msv_status msv_encode_residues(const char* letters, size_t n, uint8_t* codes_out);

/* ---------------------------------------------------------------------------------------- */
/* Device: the hot path -- replaces MSV_HMM::parallel_run_on_sequence (MSV_HMM.cpp:269-430) */
/* and its 6 OpenCL kernels (MSV_kernels.cl:1-65, MSV_spec_kernels.cl:1-50) with ONE fused   */
/* HIP kernel launch per batch.                                                              */
/* ---------------------------------------------------------------------------------------- */

/* Builds a device-resident profile from the precomputed MSV table (exactly what
 * msv_hmm_msv_scores returns).  model_length = LENG + 1. */
msv_status msv_profile_create(int device, const float* emission_scores, uint32_t model_length, float tr_B_Mk,
                              float tr_E_C, float tr_E_J, msv_profile** out);
/* Convenience: parse-side object straight to a device profile (MSV_HMM(const Profile_HMM&), MSV_HMM.hpp:19). */
msv_status msv_profile_create_from_hmm(int device, const msv_hmm* hmm, msv_profile** out);
void msv_profile_destroy(msv_profile* profile);

typedef struct msv_kernel_info {
    uint32_t model_length;     /* LENG + 1                                           */
    uint32_t lanes_per_group;  /* G: lanes that own one sequence's DP row            */
    uint32_t states_per_lane;  /* S: match states held in registers by each lane     */
    uint32_t waves_per_block;  /* 64-lane waves per workgroup                        */
    uint32_t lds_rows;         /* residue rows of the emission table staged in LDS   */
    uint32_t lds_bytes;        /* LDS used per workgroup                             */
    uint32_t blocks;           /* workgroups per launch (persistent grid)            */
    uint32_t max_length;       /* longest sequence the transition table covers        */
    int device;
    char variant[64];          /* throughput plan: batches above latency_max_n and mid_max_n */
    char latency_variant[64];  /* small-batch plan (one sequence per wave), "" if none      */
    uint32_t latency_blocks;   /* its persistent grid                                    */
    uint64_t latency_max_n;    /* batches of up to this many sequences take it            */
    char mid_variant[64];      /* mid-size plan (two sequences per wave), "" if none        */
    uint32_t mid_blocks;       /* its persistent grid                                    */
    uint64_t mid_max_n;        /* batches above latency_max_n, up to this many, take it   */
    char coop_variant[64];     /* cooperative plan (one sequence per workgroup, its row over 4 waves), "" if none */
    uint32_t coop_blocks;      /* its grid (one workgroup per CU)                          */
    uint64_t coop_max_n;       /* batches of up to this many sequences take it (before the latency plan) */
} msv_kernel_info;
msv_status msv_profile_describe(const msv_profile* profile, msv_kernel_info* out);
/* The kernel variant a batch of n sequences runs (msv_score_batch* / grid launches pick the plan by
 * batch size: latency plan, mid plan, throughput plan); "" for a null profile. */
const char* msv_profile_variant_for(const msv_profile* profile, uint64_t n);

/* The compiled kernel family (template instantiations over G, S, waves; names "msv_g<G>_s<S>_w<W>").
 * msv_profile_create picks the cheapest variant with G*S >= LENG; msv_profile_set_variant forces
 * another one (tuning / tests).  Every variant returns identical scores. */
int msv_variant_count(void);
const char* msv_variant_name(int i);
msv_status msv_profile_set_variant(msv_profile* profile, const char* name);

/* Grow the per-sequence transition table so sequences up to max_length residues can be
 * scored (default 131072). Host logf values, so the device never evaluates logf. */
msv_status msv_profile_reserve_length(msv_profile* profile, uint64_t max_length);

/* Page-locked host memory (visible to every GPU).  Residues and scores in such buffers are read and
 * written by the kernels in place (msv_score_batch: no staging copy, ~0.93 of the HBM-resident rate on
 * the BASELINE configs) -- the allocator for FFI callers that cannot reach hipHostMalloc.  Release with
 * msv_host_free.  (Any page-locked memory works the same: hipHostMalloc, hipHostRegister, torch
 * pin_memory.) */
msv_status msv_host_alloc(size_t bytes, void** out);
msv_status msv_host_free(void* ptr);

/* Host buffers in, host scores out; synchronous.  n = number of sequences; offsets has n+1
 * entries, offsets[0] may be non-zero.  scores[s] = MSV log-odds score of sequence s, exactly
 * MSV_HMM::run_on_sequence (MSV_HMM.cpp:74-113); an empty sequence scores -inf.
 * stream may be NULL (the library's own stream).  Batches of >= 4 Mi residues run as a copy/compute
 * pipeline (H2D of later pieces under the kernels of earlier ones); residues in pinned host memory
 * (hipHostMalloc, torch pin_memory) copy at full PCIe rate without runtime staging.  Pinned `scores`
 * are written by the kernels themselves through their device alias (no D2H copy). */
msv_status msv_score_batch(msv_profile* profile, const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                           float* scores, void* stream);

/* Asynchronous host-buffer scoring for a STREAM of batches (serving): enqueues the H2D of the
 * inputs on the profile's copy stream and the order, kernel and score D2H on one of its two compute
 * streams (consecutive calls alternate, so a call's kernel fills the previous one's drain tail), and
 * returns at once with a ticket; msv_profile_wait(ticket) blocks until that call's scores are in
 * `scores` and returns its kernel-latched errors.  Three staging sets, so the copies of the next calls
 * run back to back under the kernels of the earlier ones; at most 3 calls may be outstanding (a fourth
 * returns MSV_ERR_INVALID_ARGUMENT until the oldest is waited for).  The caller keeps residues/offsets
 * unchanged and does not read scores until the wait; pinned (page-locked) host buffers make the
 * copies truly asynchronous, and pinned `scores` are written by the kernel directly (no D2H; that
 * call's errors are then read from its scores: +inf = bad residue, NaN = too long).  One launch per
 * call: residues < 2^32 - 2^20 bytes. */
msv_status msv_score_batch_async(msv_profile* profile, const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                                 float* scores, uint64_t* ticket);
msv_status msv_profile_wait(msv_profile* profile, uint64_t ticket);

/* Device-resident inputs and output (e.g. hipMalloc'd or torch tensors' data pointers), enqueued
 * on `stream` (a hipStream_t, NULL = the library's stream) without a host synchronisation.
 * residues_len = bytes addressable at d_residues (must be < 2^32 per call; split larger batches).
 * d_order: optional permutation (n uint32) giving the order sequences are dequeued in
 * (e.g. longest first); NULL = input order.  Errors found by the kernel (bad residue code,
 * sequence longer than the table) are latched and returned by msv_profile_check. */
msv_status msv_score_batch_device(msv_profile* profile, const uint8_t* d_residues, uint64_t residues_len,
                                  const uint64_t* d_offsets, uint64_t n, const uint32_t* d_order, float* d_scores,
                                  void* stream);

/* Declares `stream` (a hipStream_t) as this profile's working stream until the next bind (NULL
 * unbinds): the caller guarantees it stays alive while bound.  Launches on a bound stream (and on the
 * library's own streams) skip the per-launch event that orders a counter slot's reuse across streams
 * (recorded lazily instead, only if another stream takes the slot): ~4 us less per launch, 3% of a
 * 10k-sequence 100.hmm batch.  Unbound caller streams stay correct, just with that event. */
msv_status msv_profile_bind_stream(msv_profile* profile, void* stream);

/* Synchronises `stream` and returns (then clears) the errors latched by earlier device calls. */
msv_status msv_profile_check(msv_profile* profile, void* stream);

/* Device helper: writes a longest-first dequeue order for a device CSR batch into d_order
 * (n uint32) using a counting sort on the device.  Enqueued on `stream`. */
msv_status msv_order_longest_first(msv_profile* profile, const uint64_t* d_offsets, uint64_t n, uint32_t* d_order,
                                   void* stream);

/* A GPU-parsed FASTA set (msv_fasta_read_device) scored in place: length table reserved for its
 * longest record, longest-first order, one launch, scores copied to the host (count() floats).
 * The set must live on the profile's device (else MSV_ERR_INVALID_ARGUMENT). */
msv_status msv_score_fasta_device(msv_profile* profile, const msv_fasta_device* fasta, float* scores);

/* ---- profiles x sequences grid ---------------------------------------------
 * Replaces the reference's benchmark loop over every profile for one FASTA set
 * (algorithms/benchmark_MSV.cpp:12-24,31-41: one MSV_HMM per .hmm, each scoring every sequence).
 * Every profile keeps its own compile-time kernel variant (the analog of should_specialize,
 * MSV_HMM.cpp:322-337); the launches are forked onto the profiles' own streams so that small
 * batches of different profiles run concurrently, and joined back into `stream`.
 * scores: [n_profiles][n] row-major (profile-major).  All profiles must live on one device; the
 * same profile may appear more than once (its launches then serialise).  Errors latched by the
 * kernels are reported by msv_profile_check on each profile (the host variant does that itself). */
msv_status msv_score_grid(msv_profile* const* profiles, uint32_t n_profiles, const uint8_t* residues,
                          const uint64_t* offsets, uint64_t n, float* scores, void* stream);
msv_status msv_score_grid_device(msv_profile* const* profiles, uint32_t n_profiles, const uint8_t* d_residues,
                                 uint64_t residues_len, const uint64_t* d_offsets, uint64_t n,
                                 const uint32_t* d_order, float* d_scores, void* stream);

/* ---- several devices from one host thread (SURVEY 8(b) msv_score_batch_multi, 8(e)) ----------
 * The reference has no multi-device path.  Sequences are independent, so a batch is cut into
 * contiguous shards with ~equal residue counts (a prefix-sum split that keeps the output order):
 * bounds[k] .. bounds[k+1] is shard k's sequence range (n_shards + 1 entries, bounds[0] = 0,
 * bounds[n_shards] = n).  Host-only; the torch.distributed path (one process per GPU, RCCL
 * gather) uses the same split (hmm_fasta_viterbi_amd/distributed.py). */
msv_status msv_shard_bounds(const uint64_t* offsets, uint64_t n, uint32_t n_shards, uint64_t* bounds);

/* profiles[k]: the same model created on device k (msv_profile_create_from_hmm(k, ...)).  Shard k
 * of the batch is scored on profiles[k]'s device by its own host thread (upload, longest-first
 * order, one launch, download), all shards concurrently; scores land in input order.  The same
 * device may appear more than once (its shards then share the GPU); the same HANDLE may too, and
 * then scores its shards one after another on one thread. */
msv_status msv_score_batch_multi(msv_profile* const* profiles, uint32_t n_profiles, const uint8_t* residues,
                                 const uint64_t* offsets, uint64_t n, float* scores);

/* ---- several devices from one process, scores gathered over RCCL --------------
 * A context over profiles[k] = the same model created on DISTINCT devices (rank k = profiles[k]'s
 * device; one RCCL communicator per device from ncclCommInitAll).  msv_multi_score_batch cuts the
 * batch into residue-balanced contiguous shards (msv_shard_bounds), one host thread per device uploads
 * its shard and enqueues the longest-first order and the kernel on the context's stream for that
 * device, then ONE RCCL group (ncclSend from every rank, ncclRecv into device 0's buffer at the
 * shard's offset -- exact counts, rank 0 included through a self send/recv) gathers the float scores
 * on device 0, and a single D2H returns them in input order.  A device listed twice is
 * MSV_ERR_INVALID_ARGUMENT (one rank per device); RCCL failures are MSV_ERR_RCCL.  The context
 * holds the profiles by pointer: destroy it before them. */
typedef struct msv_multi msv_multi;
msv_status msv_multi_create(msv_profile* const* profiles, uint32_t n_profiles, msv_multi** out);
msv_status msv_multi_score_batch(msv_multi* multi, const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                                 float* scores);
void msv_multi_destroy(msv_multi* multi);

/* ---- MSV filter P-values -----------------------------------------------------
 * The reference parses STATS LOCAL MSV mu/lambda (data_readers/Profile_HMM.cpp:73-94) and never
 * uses them; its README's intent is the HMMER3 filter pipeline.  This is HMMER3's formula for the
 * MSV stage: null1 score nullsc = L log(p1) + log(1 - p1), p1 = L/(L+1) (float, as p7_bg_NullOne);
 * bits = (score - nullsc) / ln 2 (float); P = Gumbel survival(bits; mu, lambda)
 * = 1 - exp(-exp(-lambda (bits - mu))), with the small-tail branch -> exp(-lambda (bits - mu)).
 * There is no reference implementation to pin against ("parity unpinned"); the device and host
 * paths agree with a float64 restatement in tests/.  Empty sequences (score -inf) give P = 1. */
msv_status msv_pvalues(const float* scores, const uint64_t* offsets, uint64_t n, float mu, float lambda,
                       double* pvalues);
msv_status msv_pvalues_device(int device, const float* d_scores, const uint64_t* d_offsets, uint64_t n, float mu,
                              float lambda, double* d_pvalues, void* stream);

/* MSV filter on the device: the P-value of every score (the formula above, written to d_pvalues when it
 * is not NULL) and the indices of the sequences with P <= threshold written to d_selected (n uint32 of
 * room), their number to *d_count (one device uint32).  d_order (NULL or a permutation of 0..n-1, e.g.
 * msv_order_longest_first's) is the order the survivors are listed in, exactly (a stable compaction, two
 * launches): with the longest-first permutation the Viterbi launch dequeues its survivors longest first
 * and its drain tail is its shortest ones.  The survivors list feeds
 * msv_vit_score_batch_device directly (no host round trip).  `stream` must not be NULL
 * (MSV_ERR_INVALID_ARGUMENT): the profiles' calls take NULL as their own non-blocking stream, which the
 * legacy null stream does not order against, so pass the same explicit stream to the calls it chains. */
msv_status msv_filter_select_device(int device, const float* d_scores, const uint64_t* d_offsets,
                                    const uint32_t* d_order, uint64_t n, float mu, float lambda, double threshold,
                                    double* d_pvalues, uint32_t* d_selected, uint32_t* d_count, void* stream);

/* ---- Viterbi stage -----------------------------------------------------------
 * The reference parses everything a Viterbi filter needs -- insert_emissions and the 7 transitions
 * per node (data_readers/Profile_HMM.hpp:28-29, Profile_HMM.cpp:107-120) and STATS LOCAL VITERBI
 * (Profile_HMM.cpp:86-87) -- and never uses it; its README (README.md:2-3) names the Viterbi algorithm
 * as the project's point.  This stage scores HMMER3's generic local Viterbi (p7_GViterbi's recurrence,
 * multihit local mode) over that parse, with the MSV path's own specials (MSV_HMM.cpp:49-64):
 *   M(i,k) = max(M(i-1,k-1)+tMM, I(i-1,k-1)+tIM, D(i-1,k-1)+tDM, B(i-1)+tr_B_Mk) + match[r][k]
 *   I(i,k) = max(M(i-1,k)+tMI, I(i-1,k)+tII) + insert[r][k]        k < LENG (no I at node LENG)
 *   D(i,k) = max(M(i,k-1)+tMD, D(i,k-1)+tDD)
 *   E = max_k M(i,k) (local exits; D(i,LENG) never exceeds it); J, C, N, B and the final C(L) + tr_move
 *   exactly as MSV_HMM::run_on_sequence (MSV_HMM.cpp:100-112, per-length tr_loop / tr_move).
 * Transition t of node k is read from transition_scores[k * 7 + t] (order m->m m->i m->d i->m i->i d->m
 * d->d, as the .hmm file) for nodes 1 .. LENG-1 only: node 0 (B) enters through tr_B_Mk, node LENG has
 * no successor -- so the '*' entries (which the reference parses as probability 1) are never read.
 * There is no reference implementation ("parity unpinned"): the device scores equal the serial
 * restatement in oracle/ bit for bit, and the stage is pinned statistically against every profile's
 * STATS LOCAL VITERBI (tests/). */
typedef struct msv_vit_profile msv_vit_profile;

typedef enum msv_insert_mode {
    MSV_INSERTS_ZERO = 0,    /* HMMER3's convention: insert emissions score 0 (background)          */
    MSV_INSERTS_LOG_ODDS = 1 /* logf(insert_emissions[k][r] / background[r]) of the reference's parse */
} msv_insert_mode;

/* Score tables of the Viterbi stage from a parsed profile (model_length = M = LENG + 1):
 * match_scores [20][M] (== msv_hmm_msv_scores' table), insert_scores [20][M] (0, or the log-odds),
 * transition_scores [M][7] = logf(parsed probability).  Any output pointer may be NULL. */
msv_status msv_hmm_viterbi_scores(const msv_hmm* hmm, int insert_mode, float* match_scores, float* insert_scores,
                                  float* transition_scores, float* tr_B_Mk, float* tr_E_C, float* tr_E_J);

/* The serial CPU Viterbi of one sequence (this library's own restatement, two rolling rows; the
 * reference-shaped Viterbi_HMM::run_on_sequence in msv_hmm.hpp).  codes 0..19; a code >= 20 gives
 * MSV_ERR_BAD_RESIDUE.  insert_scores NULL = zero insert scores. */
msv_status msv_vit_cpu_score(const float* match_scores, const float* insert_scores, const float* transition_scores,
                             uint32_t model_length, float tr_B_Mk, float tr_E_C, float tr_E_J, const uint8_t* codes,
                             uint64_t L, float* score);

/* Device-resident Viterbi profile.  insert_scores NULL = zero insert scores (MSV_INSERTS_ZERO).  Every
 * transition score the recurrence reads (nodes 1 .. LENG-1) must be <= 0, as log-probabilities are
 * (MSV_ERR_INVALID_ARGUMENT otherwise: the kernel relies on it to leave D(LENG) out of E).
 * Threading, as msv_profile: one host thread at a time; from it, device launches may go to any streams
 * (each takes its own dequeue-counter slot, reused only after that slot's previous launch), so
 * launches of one profile on different streams may overlap. */
msv_status msv_vit_profile_create(int device, const float* match_scores, const float* insert_scores,
                                  const float* transition_scores, uint32_t model_length, float tr_B_Mk, float tr_E_C,
                                  float tr_E_J, msv_vit_profile** out);
msv_status msv_vit_profile_create_from_hmm(int device, const msv_hmm* hmm, int insert_mode, msv_vit_profile** out);
void msv_vit_profile_destroy(msv_vit_profile* profile);
msv_status msv_vit_profile_reserve_length(msv_vit_profile* profile, uint64_t max_length);

typedef struct msv_vit_info {
    uint32_t model_length;    /* LENG + 1                                                   */
    uint32_t states_per_lane; /* S: one sequence per 64-lane wave, 64 * S >= LENG             */
    uint32_t transitions_in_registers; /* of the 7 per-slot transition arrays (the rest in LDS) */
    uint32_t match_in_lds;    /* match scores staged in LDS (else read from L2 every row)    */
    uint32_t insert_scores;   /* informative insert scores (read from L2)                    */
    uint32_t waves_per_block;
    uint32_t blocks;          /* persistent grid of a full launch                           */
    uint32_t lds_bytes;
    uint32_t max_length;
    int device;
    char variant[64];
    /* appended fields (append-only: the round-4 prefix above keeps its offsets) */
    uint32_t scratch_bytes;   /* private (scratch) memory per lane of the variant's kernel: spills or
                                 arrays the compiler could not keep in registers (0 for a healthy variant) */
    uint32_t waves_per_sequence; /* 1, or a team of waves sharing one sequence's row (vit_team.hip) */
} msv_vit_info;
msv_status msv_vit_profile_describe(const msv_vit_profile* profile, msv_vit_info* out);
int msv_vit_variant_count(void);
const char* msv_vit_variant_name(int i);
/* Force one compiled variant (tuning / tests); every variant returns identical scores. */
msv_status msv_vit_profile_set_variant(msv_vit_profile* profile, const char* name);

/* Device-resident batch, enqueued on `stream` (NULL = the library's stream).  d_select (optional): the
 * indices of the sequences to score, *d_select_count of them when d_select_count is given (a device
 * uint32, e.g. msv_filter_select_device's d_count), else n of them; NULL = every sequence.  Scores are
 * written at the sequence's index in d_scores (others untouched).  An empty sequence scores -inf; errors
 * (bad residue: +inf score, too long: NaN, a d_select entry >= n: skipped) are latched for
 * msv_vit_profile_check. */
msv_status msv_vit_score_batch_device(msv_vit_profile* profile, const uint8_t* d_residues, uint64_t residues_len,
                                      const uint64_t* d_offsets, uint64_t n, const uint32_t* d_select,
                                      const uint32_t* d_select_count, float* d_scores, void* stream);
/* As msv_profile_bind_stream: `stream` is this profile's working stream until the next bind (NULL
 * unbinds), kept alive by the caller while bound; launches on it skip the per-launch slot event. */
msv_status msv_vit_profile_bind_stream(msv_vit_profile* profile, void* stream);
/* Host buffers in and out, synchronous (every sequence scored); reports only its own errors (errors of
 * earlier device launches stay latched for msv_vit_profile_check). */
msv_status msv_vit_score_batch(msv_vit_profile* profile, const uint8_t* residues, const uint64_t* offsets, uint64_t n,
                               float* scores, void* stream);
msv_status msv_vit_profile_check(msv_vit_profile* profile, void* stream);

/* The filter pipeline on host buffers (HMMER3's MSV -> Viterbi cascade): MSV scores of every sequence
 * (msv_score_batch_device, longest-first), P-values against (msv_mu, msv_lambda), then the Viterbi
 * score of every sequence with P <= F1; msv_scores[n], passed[n] (0/1) and vit_scores[n] (-inf where not
 * passed) are written, *n_passed = the survivors' count.  Everything between upload and download
 * stays on the device.  msv and vit must live on one device. */
msv_status msv_vit_filter_batch(msv_profile* msv, msv_vit_profile* vit, const uint8_t* residues,
                                const uint64_t* offsets, uint64_t n, float msv_mu, float msv_lambda, double F1,
                                float* msv_scores, uint8_t* passed, float* vit_scores, uint64_t* n_passed);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MSV_H_ */
