// RNS polynomial primitive layer (L1 in SURVEY.md §1).
//
// Two implementations exist and are bit-for-bit interchangeable:
//   * csrc/hip/prims_hip.hip  -- the product: hand-written gfx950 kernels;
//   * oracle/prims_ref.c      -- the CPU oracle (test infrastructure only).
// The host CKKS layer (csrc/core/*.cpp) is compiled against this interface
// once per backend.  The product library never contains the oracle.
//
// Data layout (HBM): a polynomial with L limbs is L contiguous rows of n u64
// residues, limb-major: limb i at base + i*n.  A ciphertext is two such
// polynomials back to back (c0 rows, then c1 rows).  Limb i of a polynomial
// uses prime index  i < split ? i : pbase + (i - split)  in the context's
// prime table [q_0 .. q_L, p_0 .. p_{K-1}] (the "limb map").
//
// Every primitive is enqueued on the backend's stream; the host observes
// results only through sfp_d2h (which synchronises).
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFP_MAX_LIMBS 96
#define SFP_MAX_WSUM 80

typedef struct sfp_dev sfp_dev;

typedef struct {
    uint32_t count;   // number of limbs
    uint32_t split;   // limbs [0, split) -> primes base, base + stride, ...
    uint32_t pbase;   // limbs [split, count) -> primes pbase, pbase + stride, ...
    uint32_t base;    // (0 unless addressing a run that starts mid-table)
    uint32_t stride;  // prime step between consecutive limbs; 0 or 1 = contiguous.
                      // A limb-sharded rank r of W holds primes r, r + W, ...
} sfp_limbs;

static inline uint32_t sfp_prime_of(sfp_limbs m, uint32_t i) {
    const uint32_t st = m.stride ? m.stride : 1;
    return i < m.split ? m.base + i * st : m.pbase + (i - m.split) * st;
}

// Tables the host computes once per context (identical for both backends).
typedef struct {
    uint32_t logn;
    uint32_t nprimes;       // L+1+K
    const uint64_t* primes; // nprimes
    // per prime, n entries each (bit-reversed psi powers, OpenFHE/SEAL layout)
    const uint64_t* psi_rev;        // [nprimes][n]
    const uint64_t* psi_rev_shoup;  // [nprimes][n]
    const uint64_t* ipsi_rev;       // [nprimes][n]
    const uint64_t* ipsi_rev_shoup; // [nprimes][n]
    const uint64_t* n_inv;          // [nprimes]
    const uint64_t* n_inv_shoup;    // [nprimes]
} sfp_tables;

// Base-conversion table for fast basis extension from a source set S of
// primes to a target set T (Halevi-Polyakov-Shoup / OpenFHE "PartQlHat"):
//   y_i  = x_i * shat_inv[i] mod s_i                 (i in S)
//   out_t = sum_i y_i * shat_mod[i][t] mod t          (t in T)
// where shat = prod(S) / s_i.  Lives in backend memory (sfp_upload_conv).
typedef struct sfp_conv sfp_conv;

// ---- lifetime / memory --------------------------------------------------
sfp_dev* sfp_create(int device, const sfp_tables* t);
void sfp_destroy(sfp_dev* d);
const char* sfp_backend_name(void);
void* sfp_alloc(sfp_dev* d, size_t bytes);
void sfp_free(sfp_dev* d, void* p);
void sfp_h2d(sfp_dev* d, void* dst, const void* src, size_t bytes);
void sfp_d2h(sfp_dev* d, void* dst, const void* src, size_t bytes);
void sfp_d2d(sfp_dev* d, void* dst, const void* src, size_t bytes);
void sfp_zero(sfp_dev* d, void* dst, size_t bytes);
void sfp_sync(sfp_dev* d);
// Returns 0 if no asynchronous error is pending; otherwise an error string.
const char* sfp_last_error(sfp_dev* d);

// ---- NTT ----------------------------------------------------------------
// In-place negacyclic NTT of every limb (forward: coefficient -> evaluation
// at psi^(2*brev(k)+1); inverse includes the 1/n factor).
void sfp_ntt(sfp_dev* d, uint64_t* p, sfp_limbs m, int inverse);

// ---- elementwise ----------------------------------------------------------
void sfp_add(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m);
void sfp_sub(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m);
void sfp_neg(sfp_dev* d, uint64_t* out, const uint64_t* a, sfp_limbs m);
void sfp_mul(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m);
// out = a * b + c  (pointwise)
void sfp_mul_add(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b,
                 const uint64_t* c, sfp_limbs m);
// out[i] = a[i] * k[limb] (k: host array of m.count residues)
void sfp_mul_const(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* k,
                   sfp_limbs m);
// out[i] = a[i] + k[limb]
void sfp_add_const(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* k,
                   sfp_limbs m);
// Ciphertext tensor: d0 = a0 b0, d1 = a0 b1 + a1 b0, d2 = a1 b1
void sfp_tensor(sfp_dev* d, uint64_t* d0, uint64_t* d1, uint64_t* d2, const uint64_t* a0,
                const uint64_t* a1, const uint64_t* b0, const uint64_t* b1, sfp_limbs m);
// out = sum_j ins[j] * k[j][limb]  (+ k0[limb] if k0 != NULL), j < nin <= SFP_MAX_WSUM.
// ins: host array of device pointers; k: host array nin x m.count.
void sfp_lin_wsum(sfp_dev* d, uint64_t* out, const uint64_t* const* ins, const uint64_t* k,
                  uint32_t nin, sfp_limbs m);
// Several weighted sums of the same ciphertext inputs in one pass (the
// Chebyshev leaves): for o < nout, p in {0, 1}:
//   out + o*out_stride + p*poly_stride  =  sum_j in_p[j] * k[o][j][limb]
// in0/in1: host arrays of nin device pointers (c0 / c1 of each input),
// nin <= SFP_MAX_WSUM; k: host array nout x nin x m.count.
void sfp_lin_wsum_multi(sfp_dev* d, uint64_t* out, size_t out_stride, size_t poly_stride,
                        const uint64_t* const* in0, const uint64_t* const* in1, uint32_t nin,
                        const uint64_t* k, uint32_t nout, sfp_limbs m);

// out = sum_j a[j] * b[j]  (pointwise products summed, nin <= SFP_MAX_WSUM).
// a, b: host arrays of device pointers.
void sfp_mac_plain(sfp_dev* d, uint64_t* out, const uint64_t* const* a, const uint64_t* const* b,
                   uint32_t nin, sfp_limbs m);
// Both polynomials of a ciphertext sum at once (each plaintext read once):
// out0 = sum_j a0[j] * b[j], out1 = sum_j a1[j] * b[j]  (nin <= SFP_MAX_WSUM).
void sfp_mac_plain2(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* const* a0,
                    const uint64_t* const* a1, const uint64_t* const* b, uint32_t nin, sfp_limbs m);
// ng such sums over the SAME ciphertexts (a0, a1) with their own plaintexts
// b[g * nin + j]: out0[g] / out1[g], g < ng <= SFP_MAC_MULTI_G, nin <=
// SFP_MAC_MULTI_N -- the giant steps of one baby-step set, each ciphertext
// row read once for all of them.  The same residues as ng sfp_mac_plain2
// calls.  Returns 0, or -1 (shape unsupported: the caller runs those calls).
#define SFP_MAC_MULTI_G 8
#define SFP_MAC_MULTI_N 32
int sfp_mac_plain2_multi(sfp_dev* d, uint64_t* const* out0, uint64_t* const* out1, const uint64_t* const* a0,
                         const uint64_t* const* a1, const uint64_t* const* b, uint32_t nin, uint32_t ng,
                         sfp_limbs m);

// ---- automorphism ----------------------------------------------------------
// out = sigma_g(in) in the evaluation domain (g odd, < 2n); out != in.
void sfp_automorph(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t galois, sfp_limbs m);

// ---- rescale ------------------------------------------------------------------
// in: ell limbs (evaluation domain, limb map identity); out: ell-1 limbs,
//   out_i = (in_i - [in_last]_{q_i}) * q_last^{-1} mod q_i   (in_last taken in
//   coefficient domain with the rounding offset floor(q_last/2)).
// qlinv: host array ell-1 of q_last^{-1} mod q_i.  npoly polynomials (stride
// in_stride / out_stride u64) are processed.
void sfp_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t ell, const uint64_t* qlinv,
                 uint32_t npoly, size_t in_stride, size_t out_stride);
// Same, but the dropped (last) row is modulo prime index drop_prime instead of
// ell-1 (rows 0..ell-2 stay primes 0..ell-2): the extended-modulus
// encryption's division by q_ext.
void sfp_rescale_ext(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t ell,
                     uint32_t drop_prime, const uint64_t* qlinv, uint32_t npoly, size_t in_stride,
                     size_t out_stride);

// Rescale of a product, fused (the product is never written out):
//   sfp_mul_const_rescale: out = Rescale(in * k_i), k = host array of ell
//                          per-row residues (EvalMult(ct, double), level adjust)
//   sfp_mul_rescale:       out = Rescale(in (.) m), m = ell plaintext rows
//                          shared by the npoly polys (EvalMult(ct, pt))
// Bit-identical to sfp_mul_const / sfp_mul followed by sfp_rescale.
void sfp_mul_const_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* k,
                           uint32_t ell, const uint64_t* qlinv, uint32_t npoly, size_t in_stride,
                           size_t out_stride);
void sfp_mul_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* m, uint32_t ell,
                     const uint64_t* qlinv, uint32_t npoly, size_t in_stride, size_t out_stride);

// ---- basis conversion / key switching ----------------------------------------
// Upload a conversion table: ns source primes (prime indices src_idx), nt
// target primes (dst_idx) written to output rows dst_row[t] (NULL: row t);
// shat_inv[ns], shat_mod[ns][nt].
sfp_conv* sfp_upload_conv(sfp_dev* d, uint32_t ns, const uint32_t* src_idx, uint32_t nt,
                          const uint32_t* dst_idx, const uint32_t* dst_row,
                          const uint64_t* shat_inv, const uint64_t* shat_mod);
void sfp_free_conv(sfp_dev* d, sfp_conv* c);
// Fast base conversion in the COEFFICIENT domain: src has ns rows; target t
// is written to dst row dst_row[t].
void sfp_conv_apply(sfp_dev* d, uint64_t* dst, const uint64_t* src, const sfp_conv* c);
// Centred conversion (source values taken in (-s_i/2, s_i/2], as ModDown)
// to the first nt_use targets only.
void sfp_conv_apply_centered(sfp_dev* d, uint64_t* dst, const uint64_t* src, const sfp_conv* c,
                             uint32_t nt_use);

// Hybrid key-switch ModUp of every digit (evaluation domain in and out).
//   in   : ell limbs (limb map identity), evaluation domain.
//   ext  : beta = ceil(ell/alpha) extended polys of ell+K rows each (stride
//          (ell+K)*n; row t < ell is prime t, row ell+k is prime Lq+k).  Rows
//          of digit j's own range [j*alpha, min((j+1)*alpha, ell)) are copies
//          of `in`; all others are NTT(Conv_j(INTT(in[digit j]))), with
//          convs[j] writing rows by its dst_row table.
//   scratch: ell*n words.
void sfp_modup(sfp_dev* d, uint64_t* ext, const uint64_t* in, uint32_t ell, uint32_t K,
               uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, uint64_t* scratch);

// ModUp fused with the key inner product (one key switch's ModUp + inner
// product without the extended digits' round trip through HBM): the same
// acc0 / acc1 as sfp_modup followed by sfp_ks_inner_fold (fold0 != NULL),
// sfp_ks_inner_acc (accum) or sfp_ks_inner -- except that the rows
// t >= inv_from (the P rows: ell; with the dropped q row: ell - 1; UINT32_MAX:
// none) leave after the first (ROW) pass of ModDown's inverse NTT, so the
// ModDown that follows is called with row_done = 1.  ext: beta * (ell+K) * n
// words of scratch (the COL-pass intermediate), scr: ell * n words.  Returns
// -1 (and does nothing) where the backend has no fused form -- rings of one
// NTT tile, SFHE_KS_FUSE=0, the oracle -- and the caller runs the unfused prims.
int sfp_modup_inner(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* in, uint32_t ell, uint32_t K,
                    uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key,
                    const uint64_t* fold0, const uint64_t* fold1, uint64_t fold_k, int accum, uint32_t inv_from,
                    uint64_t* ext, uint64_t* scratch);
// sfp_modup_inner in two halves (the same launches): phases 1 = the ModUp
// (INTT of `in` into scratch, the digits' conversions and forward COL pass
// into ext), 2 = the fused ROW pass + inner product reading ext and `in`
// (the same ext / scratch / in as its phase 1), 3 = both; 0 = only report
// whether the fused form exists (0) or not (-1).  Independent key switches
// run their phase 1 as batched ops, then their accumulating phase 2 in turn.
int sfp_modup_inner_phase(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* in, uint32_t ell, uint32_t K,
                          uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key,
                          const uint64_t* fold0, const uint64_t* fold1, uint64_t fold_k, int accum,
                          uint32_t inv_from, uint64_t* ext, uint64_t* scratch, int phases);

// Build (and cache) whatever per-level tables the fused ModUp of `ell` limbs
// needs, outside any sort: the context calls it for every level at key
// generation (built lazily, each level's upload drained the device inside
// the first sort).  No-op where no fused form exists (the oracle).
void sfp_modup_prepare(sfp_dev* d, const sfp_conv* const* convs, uint32_t ell, uint32_t K, uint32_t alpha);

// Key inner product:  acc0 = sum_j ext_j * kb_j,  acc1 = sum_j ext_j * ka_j
//   ext  : beta extended polys, each (ell+K) limbs, stride ext_stride.
//   key  : beta digits, each [b rows (Lq+K)][a rows (Lq+K)]; ext limb t maps to
//          key row t (t < ell) or Lq + (t - ell).
void sfp_ks_inner(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                  size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                  uint32_t Lq);
// sfp_ks_inner of the extended digits under the automorphism X -> X^gal: ext
// is read at the source index sfp_automorph maps each coefficient from, as if
// the digits had been permuted first (a hoisted rotation: the permuted copy
// of its digits is never written).
void sfp_ks_inner_aut(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                      size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                      uint32_t Lq, uint32_t gal);
// Key inner product times a plaintext in the extended basis, accumulated
// (double hoisting: a hoisted rotation's product with a diagonal before its
// ModDown, EvalRotMultAddHoisted):
//   acc_p (+)= pm (.) sum_j ext_j * key_p,j   per ext limb, pm: ell+K rows
//   (the plaintext's q rows then its P rows, evaluation domain).
void sfp_ks_inner_mul(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                      size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                      uint32_t Lq, const uint64_t* pm, int accum);
// sfp_ks_inner_mul of the digits under X -> X^gal (as sfp_ks_inner_aut)
void sfp_ks_inner_mul_aut(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                          size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                          uint32_t Lq, const uint64_t* pm, int accum, uint32_t gal);
// sfp_ks_inner accumulating: acc0 += sum_j ext_j * kb_j, acc1 += sum_j ext_j * ka_j
// (the key switches of a rotation sum share one ModDown, EvalRotateSum).
void sfp_ks_inner_acc(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                      size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                      uint32_t Lq);

// ModDown of both key-switch accumulators:
//   out_p,i (+)= (acc_p,i - NTT(Conv_{P->Q}(INTT(acc_p,P)))_i) * pinv_i,
//   with the P->Q conversion on centred residues (zero-mean rounding error).
//   acc : two polys of ell+K rows (q rows then P rows, evaluation domain),
//         acc_1 = acc + acc_stride; their P rows are destroyed.
//   add0/add1: accumulate into out0/out1 instead of overwriting.
//   pinv: host array ell of P^{-1} mod q_i.  scratch: 2*ell*n words.
//   row_done: the P rows already had their inverse NTT's first pass
//   (sfp_modup_inner with inv_from = ell).
void sfp_moddown2(sfp_dev* d, uint64_t* out0, uint64_t* out1, uint64_t* acc, size_t acc_stride,
                  uint32_t ell, uint32_t K, uint32_t Lq, const sfp_conv* c, const uint64_t* pinv,
                  int add0, int add1, uint64_t* scratch, int row_done);

// sfp_ks_inner that also folds the relinearised polys' last q row into the
// accumulators: acc_p,l += fold_k * fold_p,l  (l = ell-1, fold_k = P mod q_l),
// the input sfp_moddown_rescale expects.
void sfp_ks_inner_fold(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                       size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell,
                       uint32_t K, uint32_t Lq, const uint64_t* fold0, const uint64_t* fold1,
                       uint64_t fold_k);

// ModDown + add + rescale in one conversion (EvalMult's relinearisation and
// its rescale).  With acc from sfp_ks_inner_fold(fold = d0, d1), l = ell-1:
//   s_p,i = d_p,i + ModDown(acc_p)_i  (i < l),   s_p,l = ModDown(acc_p)_l
//   out_p = Rescale(s_p)  (l rows at out0 / out1)
// Bit-identical to sfp_moddown2(add) + sfp_rescale on unfolded accumulators:
// the dropped row's coefficients r = (INTT(acc_l) - conv_l) P^-1 come out of
// the conversion, and out_i = (acc_i - NTT(conv_i + P [r]_i)) (P q_l)^-1
// + d_i q_l^-1 needs one NTT instead of two.
//   pinv[i] = P^-1, pmod[i] = P mod q_i (i < ell);  qlinv[i] = q_l^-1 mod q_i
//   (i < l).  acc is destroyed.  scratch: 2*l*n words.  row_done: rows
//   [l, ell+K) already had their inverse NTT's first pass (inv_from = l).
void sfp_moddown_rescale(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* d0,
                         const uint64_t* d1, uint64_t* acc, size_t acc_stride, uint32_t ell,
                         uint32_t K, uint32_t Lq, const sfp_conv* c, const uint64_t* pinv,
                         const uint64_t* pmod, const uint64_t* qlinv, uint64_t* scratch, int row_done);

// EvalMult(ct, ct) end to end from its operands (a0, a1) and (b0, b1) (ell
// rows each, evaluation domain): the tensor, the relinearisation with `key`
// and the rescale -- bit-identical to sfp_tensor followed by sfp_modup +
// sfp_ks_inner_fold (fold_k = pmod[ell-1]) + sfp_moddown_rescale, with the
// tensor's three products formed inside those passes (never written out).
// out0 / out1: ell - 1 rows.  acc: 2 (ell+K) n words, ext: beta (ell+K) n,
// scratch: 2 ell n.  Returns -1 (nothing done) where the backend has no fused
// form (the caller runs the unfused prims).
int sfp_mult_relin_rescale(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* a0, const uint64_t* a1,
                           const uint64_t* b0, const uint64_t* b1, uint32_t ell, uint32_t K, uint32_t Lq,
                           uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key, const sfp_conv* c,
                           const uint64_t* pinv, const uint64_t* pmod, const uint64_t* qlinv, uint64_t* acc,
                           uint64_t* ext, uint64_t* scratch);

// ---- sampling (counter-based, deterministic) ------------------------------------
// Uniform residues mod each limb's prime: value for (limb, i) is derived from
// splitmix64(seed, stream-id = prime index, i); identical on every backend.
void sfp_sample_uniform(sfp_dev* d, uint64_t* p, sfp_limbs m, uint64_t seed);
// Load signed coefficients (same for every limb) reduced mod each prime.
void sfp_load_i64(sfp_dev* d, uint64_t* p, const int64_t* coeffs, sfp_limbs m);

// ---- CKKS encoding on the device ------------------------------------------------
// The host encoder's tables, uploaded once per device: rot[j] = 5^j mod 2n
// (j < n/2) and ksi[k] = exp(2 pi i k / 2n) as (re, im) pairs (k <= 2n).
void sfp_encode_setup(sfp_dev* d, const uint64_t* rot, const double* ksi);
// p (rows of map m, COEFFICIENT domain) = the residues of the encoding of
// `nvals` slot values (host array: doubles when `real`, else (re, im) pairs)
// zero-padded to `slots`: the special inverse FFT, packed sparsely (gap
// n / (2 slots)), each coefficient round(u * scale).  Bit-identical to the
// host encoder (core/encoder.cpp ckks_encode) followed by sfp_load_i64,
// provided no coefficient needs the encoder's 2^shift range extension (the
// caller checks |value| * scale < 2e18).  No host synchronisation (the values
// travel through the argument ring), so it may run inside a graph capture.
// scratch: 2 * slots words.
void sfp_encode(sfp_dev* d, uint64_t* p, const double* vals, uint32_t nvals, int real, uint32_t slots,
                double scale, sfp_limbs m, uint64_t* scratch);
// `count` encodings at once (one slot count, value count and real-ness):
// rows dst + b * dstStride <- the encoding of vals + b * nvals (* 2 when
// complex), each as sfp_encode; scratch: count * 2 * slots words
void sfp_encode_batch(sfp_dev* d, uint64_t* dst, size_t dstStride, const double* vals, uint32_t nvals,
                      uint32_t count, int real, uint32_t slots, double scale, sfp_limbs m, uint64_t* scratch);
// sfp_ntt of `count` row sets p + b * stride (each the rows of map m), one launch per pass
void sfp_ntt_batch(sfp_dev* d, uint64_t* p, size_t stride, uint32_t count, sfp_limbs m, int inverse);

// ---- lanes: independent in-order queues (HIP streams) ----------------------------
// Every prim launches on the current lane.  Work on different lanes may run
// concurrently; order it with events.  The oracle has one synchronous lane
// and treats every call below as satisfied.
#define SFP_MAX_LANES 16  // (real lanes <= 8; the rest: a batched op's virtual lanes)
typedef struct sfp_event sfp_event;
int sfp_lanes(sfp_dev* d);
void sfp_set_lane(sfp_dev* d, int lane);
int sfp_get_lane(sfp_dev* d);
// Event at the current end of the current lane.
sfp_event* sfp_event_record(sfp_dev* d);
// The current lane waits (device-side) for `e`; no-op for an event of this lane.
void sfp_event_wait(sfp_dev* d, const sfp_event* e);
int sfp_event_done(sfp_dev* d, const sfp_event* e);
void sfp_event_free(sfp_dev* d, sfp_event* e);
// Lane `waiter` waits for everything enqueued so far on lane `waitee`.
void sfp_lane_wait(sfp_dev* d, int waiter, int waitee);

// ---- stacked launches ----------------------------------------------------------
// Between sfp_stack_begin and sfp_stack_end the lanes' work is recorded per
// lane and issued at the end (or at any host synchronisation) on lane 0's
// stream: each lane's work in its own order, every event wait after its
// record, and two lanes' next launches of the same kernel (NTT pass, fused
// key-switch pass, base conversion, ModDown+rescale conversion) over
// different rows merged into ONE launch -- the sort's batches, which run the
// same op sequence on two lanes, take half the launches.  Results are
// bit-identical.  No-op for the oracle, with serialised lanes, or with
// SFHE_STACK=0.  sfp_stack_stats: launches issued merged (pairs) / alone.
void sfp_stack_begin(sfp_dev* d);
void sfp_stack_end(sfp_dev* d);
void sfp_stack_stats(sfp_dev* d, uint64_t* merged, uint64_t* single);

// Batched ops (the same mechanism for independent ops of ONE host lane: the
// Chebyshev PS's products of one tree level, a polynomial's powers of one
// depth).  sfp_batch_begin(d, count) returns 1 if batching is on; the host
// then issues op i after sfp_batch_lane(d, i) and calls sfp_batch_end, which
// issues everything on the caller's lane, identical launches of different ops
// merged into one (up to eight; four for the element-wise kernels).  The ops' buffers must stay allocated until
// sfp_batch_end (their launches are issued there).  Returns 0 (the ops run as
// issued) for the oracle, with SFHE_BATCH=0 or inside a stacked lane region.
// Serialised lanes (sfp_serialize) still batch: a profiling sort then issues
// the same merged launches as the captured sort, each timed as ONE launch
// carrying the bytes of every op merged into it.
#define SFP_BATCH_MAX 8
int sfp_batch_begin(sfp_dev* d, uint32_t count);
void sfp_batch_lane(sfp_dev* d, uint32_t i);
void sfp_batch_end(sfp_dev* d);

// ---- multi-process limb sharding (one process per GPU) --------------------------
// Collectives over the ranks of a sharded context, ordered on the current
// lane like every other primitive.  Two transports:
//   * RCCL (HIP backend, production): sfp_comm_uid on one rank, the 128-byte
//     id shared out of band (torch.distributed), sfp_comm_init_rccl on all;
//   * host callbacks (both backends; tests): the caller's allgather/bcast over
//     host memory (e.g. torch.distributed gloo), after a stream drain.
typedef void (*sfp_host_allgather_fn)(void* user, const void* send, void* recv, size_t bytes);
typedef void (*sfp_host_bcast_fn)(void* user, void* buf, size_t bytes, int root);
// 0 on success; -1 where the backend has no RCCL (the oracle)
int sfp_comm_uid(void* uid128);
int sfp_comm_init_rccl(sfp_dev* d, int rank, int world, const void* uid128);
void sfp_comm_set_host(sfp_dev* d, int rank, int world, sfp_host_allgather_fn ag, sfp_host_bcast_fn bc,
                       void* user);
// 1 when the collectives can be recorded into a graph (RCCL, or no
// communicator at all); 0 for a host transport (it synchronises)
int sfp_comm_capturable(sfp_dev* d);
// recv = world blocks of `bytes`, rank-major (recv may contain send in place)
void sfp_allgather(sfp_dev* d, const void* send, void* recv, size_t bytes);
void sfp_bcast(sfp_dev* d, void* buf, size_t bytes, int root);

// Batch groups (the sort's independent batches split over GPU groups,
// DESIGN.md §7): a second communicator joining the ranks that hold the same
// rows of different batches -- rank `group` of `groups`.  Only an all-gather;
// same transports and ordering as above.
int sfp_group_init_rccl(sfp_dev* d, int group, int groups, const void* uid128);
void sfp_group_set_host(sfp_dev* d, int group, int groups, sfp_host_allgather_fn ag, void* user);
// recv = groups blocks of `bytes`, group-major (recv may contain send in place)
void sfp_group_allgather(sfp_dev* d, const void* send, void* recv, size_t bytes);

// Collective statistics (multi-GPU attribution: the bench splits a sharded
// sort's time into compute and exchange).  sfp_comm_stats_reset zeroes the
// counters; timed != 0 also brackets every collective with events on the
// stream it runs on (eager work only: a captured collective is counted, not
// timed).  sfp_comm_stats: collectives this rank issued since the reset (the
// all-gathers and broadcasts of both communicators that moved data), the
// bytes this rank received through them, and their summed duration in ms
// (0 unless timed).  Synchronises the lanes.
void sfp_comm_stats_reset(sfp_dev* d, int timed);
void sfp_comm_stats(sfp_dev* d, uint64_t* calls, double* bytes, double* ms);

// dst row i = src row rows[i] (count rows of n words; rows: host array)
void sfp_gather_rows(sfp_dev* d, uint64_t* dst, const uint64_t* src, const uint32_t* rows, uint32_t count);

// Rescale with the dropped row supplied in coefficient form (limb sharding:
// the row's owner broadcast it):  out_p,i = (in_p,i - [last_p]_{q_i}) * qlinv_i
// for the rows of map m (evaluation domain), last_p the centred lift of the
// dropped row modulo prime drop_prime.  npoly polys: in / out / last strides.
void sfp_rescale_rows(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* last,
                      uint32_t drop_prime, sfp_limbs m, const uint64_t* qlinv, uint32_t npoly,
                      size_t in_stride, size_t out_stride, size_t last_stride);

// Key inner product with explicit maps (limb sharding): ext rows follow the
// prime map pm (pm.split Q rows then P rows); ext row t uses key row
// t < pm.split ? t : keyQ + (t - pm.split) of each digit's [b rows][a rows]
// block of key_rows rows -- or, with keyQ == SFP_KEY_ROW_BY_PRIME, the key row
// of its prime (a whole key, key_rows = Lq + K: row r is prime r).
//   accum: acc (+)= the inner product (as sfp_ks_inner_acc)
#define SFP_KEY_ROW_BY_PRIME 0xFFFFFFFFu

// Switching-key geometry (sliced keys).  By default a key digit
// is [b rows][a rows] of Lq + K rows each, row r holding prime r.  A limb-
// sharded rank keeps a slice: the `tail` Q rows of the replicated levels
// (primes 0 .. tail-1), its own dealt Q primes >= tail (first, first + world,
// ... < lq), then the K P rows, `rows` in all (pstart = rows - K):
//   row(p) = p < tail ? p : p < lq ? tail + (p - first) / world : pstart + (p - lq)
// Every key prim then reads that layout: ext row t < ell of a replicated level
// reads row t, its P rows row pstart + (t - ell), and SFP_KEY_ROW_BY_PRIME
// reads row(prime).  rows == 0: whole keys (the default).
typedef struct {
    uint32_t rows, pstart, tail, world, first, lq;
} sfp_key_geom;
void sfp_set_key_geom(sfp_dev* d, const sfp_key_geom* g);
static inline uint32_t sfp_key_row(const sfp_key_geom* g, uint32_t p) {
    if (!g->rows) return p;
    return p < g->tail ? p : p < g->lq ? g->tail + (p - g->first) / g->world : g->pstart + (p - g->lq);
}
void sfp_ks_inner_map(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                      size_t ext_stride, const uint64_t* key, uint32_t beta, sfp_limbs pm,
                      uint32_t keyQ, uint32_t key_rows, int accum);

// ---- graph capture (hipGraph) ---------------------------------------------------
// Between sfp_capture_begin and sfp_capture_end every prim enqueued on lane 0
// -- and on any lane that waited for it (sfp_lane_wait / sfp_event_wait) -- is
// recorded into a graph instead of running; the lanes must be joined back to
// lane 0 before the end.  Small host arrays the prims upload (weights, row
// tables, kernel constants) go to a per-graph device arena filled once at the
// end, so the recorded launches read immutable copies.  Any host
// synchronisation inside the region (a download, an upload, a ring wrap)
// invalidates the capture: sfp_capture_end then returns NULL and records why.
// The oracle backend has no graphs: sfp_capture_begin returns -1.
typedef struct sfp_graph sfp_graph;
int sfp_capture_begin(sfp_dev* d);
// forget the recorded error (an abandoned capture is not a device fault)
void sfp_clear_error(sfp_dev* d);
sfp_graph* sfp_capture_end(sfp_dev* d);
int sfp_capturing(sfp_dev* d);
// Enqueue the whole graph on the current lane (stream-ordered like a prim).
void sfp_graph_launch(sfp_dev* d, sfp_graph* g);
size_t sfp_graph_nodes(const sfp_graph* g);
// The graph's kernel nodes of family `fam` (SFP_FAM_*; SFP_FAM_COUNT = every
// kernel of no family, SFP_FAM_ALL = every kernel node), re-instantiated in
// their captured order as a graph of their own and replayed `reps` times,
// timed with HIP events on the current lane: the family's kernels alone,
// back to back, with exactly the captured launch parameters.  Returns 0 and
// the milliseconds per replay, the launches and the algorithmic bytes of
// their NTT passes per replay; -1 where the backend has no graphs.
int sfp_graph_family_time(sfp_dev* d, sfp_graph* g, uint32_t fam, int reps, double* ms, uint64_t* launches,
                          double* bytes);
void sfp_graph_destroy(sfp_dev* d, sfp_graph* g);

// ---- live kernel timing ---------------------------------------------------------
// Kernel families timed with events recorded on the backend's stream around
// single launches.  Algorithmic bytes per launch (minimum HBM traffic):
//   NTT pass     16 B per coefficient (read + write once; twiddles excluded)
//   CONV         8 B per source coefficient read + 8 B per target written
//   KSINNER      8 B per ext / key / accumulator word touched (k_ks_inner)
//   NTTKS        the same for k_ntt_ks (ModUp's ROW pass fused with the inner product)
// Inside a stacked region the launches are timed as issued (a merged pair is
// one launch with the bytes of both).
enum { SFP_FAM_NTT = 0, SFP_FAM_CONV = 1, SFP_FAM_KSINNER = 2, SFP_FAM_NTTKS = 3, SFP_FAM_COUNT = 4, SFP_FAM_ALL = 5 };
// Time every `period`-th launch of `fam` (0 = off); resets its counters.
void sfp_prof_set(sfp_dev* d, uint32_t fam, uint32_t period);
// Since the last sfp_prof_set: launches seen, launches timed, their summed
// duration (ms) and summed algorithmic bytes.  Synchronises the stream.
int sfp_prof_read(sfp_dev* d, uint32_t fam, uint64_t* launches, uint64_t* timed, double* ms,
                  double* bytes);
// on != 0: every lane's work goes to lane 0's stream in issue order (a valid
// order: the host issues each op after its inputs), so timed launches do not
// overlap other lanes' kernels -- per-launch durations as rocprof reports them.
void sfp_serialize(sfp_dev* d, int on);

#ifdef __cplusplus
}
#endif
