/*
 * sfhe.h -- C ABI of the MI355X CKKS rank-sort engine (drop-in boundary).
 *
 * The reference (oksuman/sorting-fhe) is C++ calling OpenFHE 1.1.4; it has
 * no FFI of its own.  Its hot path is DirectSort<N>::sort and the lbcrypto
 * calls beneath it.  Every entry point below replaces
 * one of those reference interfaces (cited per function), with plain
 * pointers, sizes and int status codes so any FFI (ctypes, cgo, JNI, N-API)
 * can bind it.  C++ callers can instead use the lbcrypto-compatible headers
 * in sorting-fhe_amd/csrc/core and csrc/algo, which wrap the same engine.
 *
 * Conventions: functions return SFHE_OK (0) or a negative SFHE_E* code;
 * sfhe_last_error() gives the message (thread-local).  Objects returned
 * through out-pointers are owned by the caller and released with the
 * matching *_free / *_destroy.  A context and everything created from it
 * must be used from one thread at a time (calls are internally serialised).
 */
#ifndef SFHE_H
#define SFHE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFHE_ABI_VERSION 3  /* bumped when a declaration or struct below changes */

#define SFHE_OK 0
#define SFHE_EINVAL (-1)   /* bad argument */
#define SFHE_ESCHEME (-2)  /* CKKS error: depth exhausted, missing key, ... */
#define SFHE_EDEVICE (-3)  /* device / backend failure */
#define SFHE_ENOTIMPL (-4) /* valid request, not implemented */

typedef struct sfhe_ctx sfhe_ctx;
typedef struct sfhe_ct sfhe_ct;
typedef struct sfhe_sorter sfhe_sorter;

/* Scaling techniques (lbcrypto::ScalingTechnique values).  FLEXIBLEAUTOEXT,
 * OpenFHE's default and therefore the reference's (it never calls
 * SetScalingTechnique), forms fresh encryptions modulo Q*q_ext and rescales
 * by q_ext; FLEXIBLEAUTO encrypts directly modulo Q. */
#define SFHE_FLEXIBLEAUTO 2
#define SFHE_FLEXIBLEAUTOEXT 3

/* Security levels (lbcrypto::SecurityLevel). */
#define SFHE_HESTD_128_CLASSIC 0
#define SFHE_HESTD_NOTSET 3

/* CCParams<CryptoContextCKKSRNS> (GenCryptoContext inputs; reference
 * tests/DirectSortTest.cpp:29-37, sort_algo.h:87-201). */
typedef struct {
    uint32_t mult_depth;
    uint32_t scaling_mod_size;  /* bits of the scaling primes (e.g. 40) */
    uint32_t first_mod_size;    /* bits of q_0 (default 60) */
    uint32_t batch_size;        /* default slot count; 0 = n/2 */
    uint32_t ring_dim;          /* 0 = smallest secure */
    int32_t security_level;     /* SFHE_HESTD_* */
    uint32_t num_large_digits;  /* HYBRID dnum; 0 = default (3) */
    int32_t device;             /* HIP device ordinal */
    uint64_t seed;              /* deterministic key / noise sampling */
    int32_t scaling_technique;  /* SFHE_FLEXIBLEAUTO[EXT]; 0 = FLEXIBLEAUTOEXT */
} sfhe_params;

int sfhe_abi_version(void);
const char* sfhe_last_error(void);
/* "hip-gfx950" for the product library. */
const char* sfhe_backend(void);
void sfhe_params_default(sfhe_params* p);

/* ---- context and keys ---------------------------------------------------
 * Replaces GenCryptoContext + Enable(...) + KeyGen + EvalMultKeyGen
 * (DirectSortTest.cpp:39-54) and EvalRotateKeyGen (:52). */
int sfhe_context_create(const sfhe_params* p, sfhe_ctx** out);
void sfhe_context_destroy(sfhe_ctx* c);
int sfhe_keygen(sfhe_ctx* c);
int sfhe_rotate_keygen(sfhe_ctx* c, const int32_t* idx, size_t count);
/* ring_dim, mult_depth, #Q primes, #P primes, dnum (any pointer may be NULL) */
int sfhe_context_info(sfhe_ctx* c, uint32_t* ring_dim, uint32_t* mult_depth, uint32_t* num_q,
                      uint32_t* num_p, uint32_t* dnum);
/* prime table [q_0..q_L, p_0..p_{K-1}] (+ q_ext under FLEXIBLEAUTOEXT) */
int sfhe_context_primes(sfhe_ctx* c, uint64_t* out, size_t cap, size_t* count);
/* Cache of encoded constant plaintexts (sort masks) across calls; default on. */
int sfhe_set_plaintext_cache(sfhe_ctx* c, int on);
/* Suppress the reference's stdout prints inside sort() (default off). */
int sfhe_set_quiet(sfhe_ctx* c, int quiet);
/* Block until queued device work is done; reports asynchronous errors. */
int sfhe_sync(sfhe_ctx* c);
/* counts[9]: keyswitch, rescale, tensor, ptmult, constmult, add, automorph,
 * ntt_limbs, wsum_terms; bytes: algorithmic HBM bytes (SURVEY §8(d) model). */
int sfhe_op_stats(sfhe_ctx* c, uint64_t* counts, double* bytes, int reset);
/* Bootstrap shapes (input level, iterations, precision) replayed from a
 * captured hipGraph so far (the first call of a shape runs eagerly, the
 * second is captured). */
int sfhe_bootstrap_graphs(sfhe_ctx* c, uint64_t* count);
/* Plaintext encodings done on the device (sfp_encode) and on the host since
 * the last sfhe_op_stats reset. */
int sfhe_encode_counts(sfhe_ctx* c, uint64_t* device, uint64_t* host);
/* Device memory held by the context's buffer pool (live and free blocks). */
int sfhe_pool_bytes(sfhe_ctx* c, uint64_t* bytes);
/* Engine contexts alive in this process (diagnostics: after every
 * sfhe_context_destroy of a process's contexts it is back to 0). */
int sfhe_live_contexts(void);
/* Live kernel timing (bench roofline; no reference counterpart): kernel
 * families SFHE_KFAM_*; every `period`-th launch of the family is bracketed
 * by HIP events on the context's stream (period 0 = off; resets counters).
 * _read synchronises and returns launches seen, launches timed, their summed
 * duration (ms) and summed algorithmic bytes (prims.h defines the model). */
#define SFHE_KFAM_NTT 0
#define SFHE_KFAM_CONV 1
#define SFHE_KFAM_KSINNER 2
#define SFHE_KFAM_NTTKS 3   /* k_ntt_ks: ModUp's ROW pass fused with the key inner product */
#define SFHE_KFAM_OTHER 4   /* (graph timing only) every kernel of no family above */
#define SFHE_KFAM_ALL 5     /* (graph timing only) every kernel */
int sfhe_kernel_timing(sfhe_ctx* c, uint32_t family, uint32_t period);
int sfhe_kernel_timing_read(sfhe_ctx* c, uint32_t family, uint64_t* launches, uint64_t* timed,
                            double* ms, double* bytes);
/* on != 0: all of the context's lanes (streams) issue on one stream, so timed
 * launches run alone, as under rocprofv3 (bench profiling leg; slower). */
int sfhe_serialize_lanes(sfhe_ctx* c, int on);
/* Stacked launches so far (no reference counterpart; prims.h sfp_stack_*):
 * the sort's two batches issue their identical ops as one launch each --
 * `merged` such pairs, `single` launches issued alone inside stacked regions. */
int sfhe_stack_stats(sfhe_ctx* c, uint64_t* merged, uint64_t* single);
/* Collective statistics of a sharded context (no reference counterpart; the
 * reference has no distributed code): sfhe_comm_stats_reset zeroes them
 * (timed != 0: every eager collective is also timed with events on its
 * stream); sfhe_comm_stats returns the collectives this rank issued since,
 * the bytes it received through them and their summed duration in ms. */
int sfhe_comm_stats_reset(sfhe_ctx* c, int timed);
int sfhe_comm_stats(sfhe_ctx* c, uint64_t* calls, double* bytes, double* ms);

/* ---- encryption ------------------------------------------------------------
 * Replaces Encryption::encryptInput (encryption.cpp:5-12, MakeCKKSPacked-
 * Plaintext + Encrypt) and DebugEncryption::getPlaintext / Decrypt
 * (:14-33).  slots = 0 uses the batch size; level > 0 encrypts lower. */
int sfhe_encrypt(sfhe_ctx* c, const double* values, size_t len, uint32_t slots, uint32_t level,
                 sfhe_ct** out);
/* writes min(cap, slots) real parts; *len = slots */
int sfhe_decrypt(sfhe_ctx* c, const sfhe_ct* ct, double* out, size_t cap, size_t* len);
void sfhe_ct_free(sfhe_ct* ct);
int sfhe_ct_clone(const sfhe_ct* ct, sfhe_ct** out);
/* Ciphertext::GetLevel / GetSlots / limb count */
int sfhe_ct_info(const sfhe_ct* ct, uint32_t* level, uint32_t* slots, uint32_t* limbs);
/* Ciphertext::SetSlots (metadata only) */
int sfhe_ct_set_slots(sfhe_ct* ct, uint32_t slots);
/* raw residues [c0 limbs][c1 limbs] (evaluation domain), 2*limbs*n words */
int sfhe_ct_download(sfhe_ctx* c, const sfhe_ct* ct, uint64_t* out, size_t cap_words);

/* ---- evaluation (CryptoContextImpl::Eval*, as called on the hot path) ---- */
int sfhe_eval_add(sfhe_ctx* c, const sfhe_ct* a, const sfhe_ct* b, sfhe_ct** out);
int sfhe_eval_sub(sfhe_ctx* c, const sfhe_ct* a, const sfhe_ct* b, sfhe_ct** out);
int sfhe_eval_add_const(sfhe_ctx* c, const sfhe_ct* a, double k, sfhe_ct** out);
int sfhe_eval_mult_const(sfhe_ctx* c, const sfhe_ct* a, double k, sfhe_ct** out);
/* EvalMult(ct, pt): pt = encode(values, slots) at a's level */
int sfhe_eval_mult_plain(sfhe_ctx* c, const sfhe_ct* a, const double* values, size_t len,
                         uint32_t slots, sfhe_ct** out);
/* EvalMultAndRelinearize / EvalMult(ct, ct) (sign.cpp:23-33) */
int sfhe_eval_mult(sfhe_ctx* c, const sfhe_ct* a, const sfhe_ct* b, sfhe_ct** out);
/* EvalRotate (rotation.h:224) */
int sfhe_eval_rotate(sfhe_ctx* c, const sfhe_ct* a, int32_t r, sfhe_ct** out);
/* sum_k EvalRotate(a[k], r[k]) with one shared ModDown (engine extension:
 * output aggregation of the giant steps of vecRotsOpt / blindRotationOptN,
 * src/sort_algo.h:342-364, 561-584, which sum individually rotated terms) */
int sfhe_eval_rotate_sum(sfhe_ctx* c, const sfhe_ct* const* a, const int32_t* r, size_t count, sfhe_ct** out);
/* CKKS bootstrapping (OpenFHE's EvalBootstrapSetup + EvalBootstrapKeyGen and
 * EvalBootstrap, as src/k-way/EvalUtils.cpp:57-86 and src/sort_algo.h:1437
 * call them): setup for ciphertexts of `slots` slots with the level budget
 * {budget_c2s, budget_s2c} (and its rotation / conjugation keys); depth =
 * the level a bootstrapped ciphertext comes out at; iterations 2 with
 * precision p = meta-bootstrapping. */
int sfhe_bootstrap_setup(sfhe_ctx* c, uint32_t budget_c2s, uint32_t budget_s2c, uint32_t slots);
int sfhe_bootstrap_depth(sfhe_ctx* c, uint32_t budget_c2s, uint32_t budget_s2c, uint32_t slots, uint32_t* depth);
int sfhe_bootstrap(sfhe_ctx* c, const sfhe_ct* a, uint32_t iterations, uint32_t precision, sfhe_ct** out);
/* EvalChebyshevSeriesPS (sort_algo.h:727-728, sign.cpp:76); c0/2 convention */
int sfhe_eval_chebyshev(sfhe_ctx* c, const sfhe_ct* x, const double* coeffs, size_t count,
                        double a, double b, sfhe_ct** out);

/* ---- hot path ----------------------------------------------------------------
 * sign(x, cc, CompositeSign, SignConfig(CompositeSignConfig(n, dg, df)))
 * (sign.cpp:635-651; n in {3, 4}). */
int sfhe_sign(sfhe_ctx* c, const sfhe_ct* x, int n, int dg, int df, sfhe_ct** out);
/* Comparison::compare (comparison.cpp:4-22): (sign(a-b)+1)/2 */
int sfhe_compare(sfhe_ctx* c, const sfhe_ct* a, const sfhe_ct* b, int n, int dg, int df,
                 sfhe_ct** out);
/* DirectSort<N>::getSizeParameters (sort_algo.h:87-201): depth and rotation
 * keys: the reference table for N in {4, 8, ..., 2048} (sorters: N <= 1024). */
int sfhe_direct_sort_params(uint32_t N, uint32_t* mult_depth, int32_t* rotations, size_t cap,
                            size_t* count);
/* Doubled-sinc Chebyshev table (generated_doubled_sinc_coeffs.h). */
int sfhe_doubled_sinc_coeffs(uint32_t N, double* out, size_t cap, size_t* count);
/* DirectSort<N> construction (sort_algo.h:74-81; encrypts the zero cache).
 * debug != 0 uses DebugEncryption, so sort() runs the reference's three
 * PRINT_PT decrypts ("as-test" timing); 0 = plain Encryption ("pure"). */
int sfhe_sorter_create(sfhe_ctx* c, uint32_t N, int debug, sfhe_sorter** out);
/* The same with the rotation-key list the DirectSort<N> constructor receives
 * (sort_algo.h:74-81, its rotIndices argument: the amounts RotationComposer
 * uses as single steps); NULL / 0 = the getSizeParameters list.  The context
 * must hold keys for them (sfhe_keygen's rotation list). */
int sfhe_sorter_create_rot(sfhe_ctx* c, uint32_t N, int debug, const int32_t* rotations, size_t nrot,
                           sfhe_sorter** out);
void sfhe_sorter_destroy(sfhe_sorter* s);
/* DirectSort<N>::sort (sort_algo.h:752-774).  Sets the input's slots to
 * the partition size as the reference does (sort_algo.h:711). */
int sfhe_sorter_sort(sfhe_sorter* s, sfhe_ct* in, int n, int dg, int df, sfhe_ct** out);
/* DirectSort<N>::constructRank (sort_algo.h:368-506) */
int sfhe_sorter_rank(sfhe_sorter* s, const sfhe_ct* in, int n, int dg, int df, sfhe_ct** out);
/* DirectSort<N>::rotationIndexCheckN (sort_algo.h:658-750) */
int sfhe_sorter_place(sfhe_sorter* s, const sfhe_ct* rank, sfhe_ct* in, sfhe_ct** out);
/* Kernel / dependency nodes of the sorter's captured sort graph (engine
 * extension, no reference counterpart): sort() runs its first call of a shape
 * eagerly, captures the second into a hipGraph and replays it from then on
 * (SFHE_GRAPH=0 keeps every sort eager; debug sorters never capture).
 * 0 while no graph exists. */
int sfhe_sorter_graph_nodes(const sfhe_sorter* s, uint64_t* nodes);
/* Roofline measurement (engine extension): the NTT kernel nodes of the
 * sorter's captured sort graph re-instantiated alone, in captured order, and
 * replayed `reps` times, timed with HIP events: *ms per replay (= the NTT
 * kernel time of one sort), *launches, *bytes (algorithmic: 16 B per
 * coefficient per pass).  SFHE_EINVAL-class error when no graph exists. */
int sfhe_sorter_graph_ntt_time(sfhe_sorter* s, int reps, double* ms, uint64_t* launches, double* bytes);
/* The same for any family SFHE_KFAM_* (OTHER: the kernels of no family, ALL:
 * every kernel node -- the sort's kernel time without lane overlap); *bytes:
 * the algorithmic bytes of the family's kernels for NTT, CONV and NTTKS
 * (sources read and targets written once), 0 for the others. */
int sfhe_sorter_graph_family_time(sfhe_sorter* s, uint32_t family, int reps, double* ms, uint64_t* launches,
                                  double* bytes);
/* DirectSort<N>::sort_hybrid1 (sort_algo.h:1213-1229): constructRank, then
 * rotationIndexCheckHybrid1 (:1067-1209, MEHP24 indicatorAdv placement,
 * mehp24_utils.cpp:166-174, :246-261).  Needs ring dimension >= 2 N^2 for
 * N <= 256 and the DirectSortH1Test keys (sfhe_hybrid1_params). */
int sfhe_sorter_sort_hybrid1(sfhe_sorter* s, sfhe_ct* in, int n, int dg, int df, sfhe_ct** out);
/* Depth and rotation keys of tests/DirectSortH1Test.cpp:36-117 for N
 * (the reference keeps them in the test; ring 2^17, HEStd_128_classic). */
int sfhe_hybrid1_params(uint32_t N, uint32_t* mult_depth, int32_t* rotations, size_t cap, size_t* count);

/* DirectSort<N>::sort_hybrid (variant 0; sort_algo.h:1049-1062) and
 * sort_hybrid2 (variant 2; :1376-1389): constructRank, then the MEHP24 matrix
 * placement on rank / N with the scaled-sinc Chebyshev indicator (hybrid2;
 * hybrid below N = 256) or the composite-sign indicator |d| < 1/2N (hybrid at
 * N >= 256: CompositeSign(3,4,2) at 256, (3,5,2) above; rotationIndexCheck-
 * Hybrid :894-1047, -Hybrid2 :1233-1374).  Needs 2 N^2 <= the ring
 * dimension for N <= 256 and the keys of sfhe_hybrid_params. */
int sfhe_sorter_sort_hybrid(sfhe_sorter* s, sfhe_ct* in, int variant, int n, int dg, int df, sfhe_ct** out);
/* the DirectSortHTest (variant 0, tests/DirectSortHTest.cpp:29-100) and
 * DirectSortH2Test (variant 2, tests/DirectSortH2Test.cpp:39-108) depth and
 * rotation keys at ring 2^17 */
int sfhe_hybrid_params(uint32_t N, int variant, uint32_t* mult_depth, int32_t* rotations, size_t cap,
                       size_t* count);
/* DirectSort<N>::rotationIndexCheck2N (sort_algo.h:587-656): placement over
 * 2N-slot blocks with the scaled sinc (rank from sfhe_sorter_rank). */
int sfhe_sorter_place_2n(sfhe_sorter* s, const sfhe_ct* rank, sfhe_ct* in, sfhe_ct** out);
/* BitonicSort<N>::sort (sort_algo.h:1421-1486): the compare-and-swap network
 * over the sorter's N slots with EvalBootstrap(ct, 2, 20) whenever the level
 * passes 29 -- needs sfhe_bootstrap_setup for N slots and the +-2^i keys the
 * sorter was created with; input values in [0, 255]. */
int sfhe_sorter_sort_bitonic(sfhe_sorter* s, sfhe_ct* in, int n, int dg, int df, sfhe_ct** out);

/* Serialized I/O (src/sort.h:31-102, src/main.cpp:9-44: the FHERMA-style file
 * set).  sfhe_save writes <dir>/cc.bin, pub.bin, mult.bin, rot.bin and, if the
 * context holds it, sk.bin; sfhe_load reads them back into a new context
 * (sk.bin optional).  Records are this engine's (magic, version, kind, context
 * fingerprint), not OpenFHE's cereal layout. */
int sfhe_save(sfhe_ctx* c, const char* dir);
int sfhe_load(const char* dir, sfhe_ctx** out);
int sfhe_ct_save(sfhe_ctx* c, const sfhe_ct* ct, const char* path);
int sfhe_ct_load(sfhe_ctx* c, const char* path, sfhe_ct** out);

/* k-way sorting network: KWayAdapter<N>::sort = kwaySort::Sorter::sorter
 * (src/kway_adapter.h:66-72, src/k-way/Sorter.cpp:284-404) over k^M = the
 * ciphertext's first slots, k in {2, 3, 5}; comparisons CompositeSign(n, dg,
 * df) with lazy bootstrapping against mult_depth (SignConfig(cfg, multDepth),
 * tests/k-way/KWaySort2Test.cpp:157 -- note that test passes (3, d_f, d_g));
 * needs sfhe_bootstrap_setup for the ciphertext's slots. */
int sfhe_kway_sort(sfhe_ctx* c, const sfhe_ct* in, int k, int M, int n, int dg, int df, uint32_t mult_depth,
                   sfhe_ct** out);
/* A persistent KWayAdapter<N> (N = k^M; k = 2: N = 4 .. 1024, k = 3: 9 .. 729,
 * k = 5: 25 .. 625): the reference's adapter object (kway_adapter.h:23-35),
 * whose sorts after the first reuse the encoded masks and bootstrapping
 * diagonals. */
typedef struct sfhe_kway sfhe_kway;
int sfhe_kway_create(sfhe_ctx* c, uint32_t N, int k, int M, sfhe_kway** out);
int sfhe_kway_run(sfhe_kway* s, const sfhe_ct* in, int n, int dg, int df, uint32_t mult_depth, sfhe_ct** out);
void sfhe_kway_destroy(sfhe_kway* s);
/* Nodes of the handle's captured sort graph (0: none yet).  The first sort of
 * a shape runs eagerly, the second is captured whole -- stages and the
 * bootstraps between them -- and later sorts replay it (SFHE_GRAPH=0: eager). */
int sfhe_kway_graph_nodes(const sfhe_kway* s, uint64_t* nodes);
/* The captured k-way sort's kernels of one family (SFHE_KFAM_*) replayed
 * alone, summed over its chain of graphs: ms per sort, launches, and their
 * algorithmic bytes (NTT, conversion and k_ntt_ks families; 0 for others).
 * No reference counterpart (bench attribution of BASELINE config 4). */
int sfhe_kway_graph_family_time(sfhe_kway* s, uint32_t family, int reps, double* ms, uint64_t* launches,
                                double* bytes);
/* KWayAdapter<N>::getSizeParameters (kway_adapter.h:41-64): batch (next power
 * of two >= N), depth 40, first modulus 60 / scale 59 bits, level budget
 * {4,4} (N <= 128) or {5,5}, the +-2^i rotation keys below N. */
int sfhe_kway_params(uint32_t N, uint32_t* batch, uint32_t* mult_depth, uint32_t* budget_c2s, uint32_t* budget_s2c,
                     int32_t* rotations, size_t cap, size_t* count);

/* Decomposer<N>::decompose (rotation.h:54-102); algo 0 NAF, 1 BNAF, 2 BINARY.
 * N in {4..1024}; writes (value, stepSize) pairs. */
int sfhe_decompose(uint32_t N, const int32_t* keys, size_t nkeys, int32_t rotation, int32_t wrapN,
                   int algo, int32_t* values, int32_t* steps, size_t cap, size_t* count);

/* ---- limb sharding (no reference counterpart: the reference
 * runs one process on one device) -------------------------------------------
 * One process per GPU; rank r of W holds the RNS limbs q_i / p_k with
 * i % W == r / k % W == r of every ciphertext level with more than the
 * replicated-tail limb count (SFHE_SHARD_TAIL, default 16; below it every
 * rank holds and computes every limb, without exchanges).  Key generation
 * and encryption run on every limb (setup) and every rank keeps whole
 * switching keys; evaluation runs on the local limbs only, with three
 * exchanges: the ModUp input (all-gather of the coefficient-form Q limbs),
 * the ModDown P limbs (all-gather) and a rescale's dropped limb (broadcast by
 * its owner), plus one all-gather where a ciphertext enters the tail.
 * Decryption and sfhe_ct_download all-gather the limbs.  Every rank makes
 * the same calls in the same order (they are collective); results are
 * bit-identical to the unsharded context.  Call once per context, after
 * sfhe_context_create and before sfhe_keygen, with the same params and seed
 * on every rank.  RCCL-sharded sorts are captured into hipGraphs with their
 * collectives; a one-rank RCCL communicator takes the sharded path too. */
/* 128-byte RCCL unique id (one rank; shared out of band).  SFHE_ENOTIMPL on
 * a backend without RCCL (the CPU oracle). */
int sfhe_comm_uid(uint8_t uid[128]);
/* RCCL communicator over xGMI (the product path). */
int sfhe_shard_rccl(sfhe_ctx* c, int rank, int world, const uint8_t uid[128]);
/* Host-memory collectives supplied by the caller (tests; any transport):
 * allgather writes world blocks of `bytes`, rank-major, into recv. */
typedef void (*sfhe_allgather_fn)(void* user, const void* send, void* recv, size_t bytes);
typedef void (*sfhe_bcast_fn)(void* user, void* buf, size_t bytes, int root);
int sfhe_shard_host(sfhe_ctx* c, int rank, int world, sfhe_allgather_fn ag, sfhe_bcast_fn bc,
                    void* user);
/* The replicated-tail limb count of a sharded context (0: unsharded). */
int sfhe_shard_tail(const sfhe_ctx* c, uint32_t* limbs);
/* Rows per digit part of this rank's switching keys: num_q + num_p for whole
 * keys; a sharded rank of world > 1 keeps only its slice (the replicated
 * tail's Q rows, its own dealt Q rows, the P rows; SFHE_KEY_SLICE=0: whole). */
int sfhe_key_rows(const sfhe_ctx* c, uint32_t* rows);

/* ---- batch groups (no reference counterpart) ------------------------------
 * DirectSort's rank and placement phases each run B independent batches
 * (reference src/sort_algo.h:438-492, 713-742, the OpenMP batch loop).  With
 * G batch groups, the ranks form G groups of W/G (each group limb-sharded
 * over its own communicator, or one unsharded rank); group g runs the
 * batches b with b % G == g and every part is all-gathered over a second
 * communicator joining the ranks that hold the same rows in different groups
 * (in-group rank r of every group).  Every rank ends with the same,
 * bit-identical result as the unsplit sort.  B not a multiple of G: every
 * group runs every batch; one group (groups == 1) runs every batch and
 * still routes each part through the communicator (single-GPU validation of
 * the collective).  Call before sfhe_keygen, with the same params and
 * seed on every rank; the calls are collective like the sharded ones. */
int sfhe_groups_rccl(sfhe_ctx* c, int group, int groups, const uint8_t uid[128]);
int sfhe_groups_host(sfhe_ctx* c, int group, int groups, sfhe_allgather_fn ag, void* user);
int sfhe_groups(const sfhe_ctx* c, int* group, int* groups);

#ifdef __cplusplus
}
#endif
#endif /* SFHE_H */
