/*
 * ORACLE -- test infrastructure only.  Never linked into the product.
 *
 * Plain-C restatement of the RNS-CKKS polynomial primitives of
 * sorting-fhe_amd/csrc/prims.h.  The reference (oksuman/sorting-fhe) takes
 * these from OpenFHE 1.1.4, which is an external dependency absent from
 * /root/reference; the algorithms restated here are the
 * published ones OpenFHE implements:
 *   - negacyclic NTT, Cooley-Tukey forward / Gentleman-Sande inverse with
 *     bit-reversed psi powers (Longa-Naehrig 2016, Alg. 1/2);
 *   - automorphism X -> X^g as an index permutation of evaluation points;
 *   - HYBRID key switching (Han-Ki 2020): ModUp by fast base conversion,
 *     digit inner product, ModDown by P;
 *   - rescale by the last prime with rounding.
 * Modular products use exact 128-bit '%' (independent of the product's
 * Barrett/Shoup code), so a bit-exact match with the HIP backend is a real
 * cross-check.  Limb loops are OpenMP-parallel (the CPU baseline).
 *
 * The host CKKS layer (csrc/core) compiled against this file gives the
 * oracle library oracle/_build/libsfhe_oracle.so (see oracle/Makefile).
 *
 * Pinning: OpenFHE's own outputs cannot be produced here, so ciphertext bits
 * are "parity unpinned" against the reference; the oracle is pinned to the
 * reference's test vectors and gates in tests/golden/ 
 * and serves as the bit-exact cross-check of the HIP kernels.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../sorting-fhe_amd/csrc/prims.h"

typedef uint64_t u64;
typedef unsigned __int128 u128;

struct sfp_dev {
    uint32_t n, logn, np;
    u64* q;
    u64 *psi, *psiS, *ipsi, *ipsiS;
    u64 *ninv, *ninvS;
    /* limb sharding: rank of world, host-callback collectives */
    int rank, world;
    sfp_host_allgather_fn ag;
    sfp_host_bcast_fn bc;
    void* user;
    /* batch groups (sfp_group_*): rank grank of gworld, host all-gather */
    int grank, gworld;
    sfp_host_allgather_fn gag;
    void* guser;
    /* the host encoder's tables (sfp_encode) */
    u64* enc_rot;
    double* enc_ksi;
    /* switching-key geometry (sfp_set_key_geom; rows == 0: whole keys) */
    sfp_key_geom kg;
    /* collective statistics (sfp_comm_stats) */
    uint64_t comm_calls;
    double comm_bytes, comm_ms;
    int comm_timed;
};

void sfp_set_key_geom(sfp_dev* d, const sfp_key_geom* g) {
    if (g)
        d->kg = *g;
    else
        memset(&d->kg, 0, sizeof d->kg);
}

struct sfp_conv {
    uint32_t ns, nt;
    uint32_t *src, *dst;
    u64 *inv, *mod;
    u64 *sprod; /* prod(S) mod dst_t */
    uint32_t *drow; /* output row of target t */
};

static inline u64 mm(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }
static inline u64 ad(u64 a, u64 b, u64 q) { u64 r = a + b; return r >= q ? r - q : r; }
static inline u64 sb(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }
static inline u64 shoup(u64 a, u64 w, u64 wp, u64 q) {
    u64 hi = (u64)(((u128)a * wp) >> 64);
    u64 r = a * w - hi * q;
    return r >= q ? r - q : r;
}
static inline uint32_t brev(uint32_t x, uint32_t bits) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}
static inline uint32_t pidx(sfp_limbs m, uint32_t i) { return sfp_prime_of(m, i); }

const char* sfp_backend_name(void) { return "oracle-c"; }

sfp_dev* sfp_create(int device, const sfp_tables* t) {
    (void)device;
    sfp_dev* d = (sfp_dev*)calloc(1, sizeof(sfp_dev));
    d->world = 1;
    d->gworld = 1;
    d->logn = t->logn;
    d->n = 1u << t->logn;
    d->np = t->nprimes;
    size_t tn = (size_t)d->np * d->n;
    d->q = (u64*)malloc(d->np * 8);
    memcpy(d->q, t->primes, d->np * 8);
    d->psi = (u64*)malloc(tn * 8);
    d->ipsi = (u64*)malloc(tn * 8);
    memcpy(d->psi, t->psi_rev, tn * 8);
    memcpy(d->ipsi, t->ipsi_rev, tn * 8);
    /* recompute the Shoup companions independently */
    d->psiS = (u64*)malloc(tn * 8);
    d->ipsiS = (u64*)malloc(tn * 8);
    d->ninv = (u64*)malloc(d->np * 8);
    d->ninvS = (u64*)malloc(d->np * 8);
    for (uint32_t p = 0; p < d->np; ++p) {
        u64 q = d->q[p];
        for (uint32_t k = 0; k < d->n; ++k) {
            size_t o = (size_t)p * d->n + k;
            d->psiS[o] = (u64)(((u128)d->psi[o] << 64) / q);
            d->ipsiS[o] = (u64)(((u128)d->ipsi[o] << 64) / q);
        }
        /* n^{-1} by Fermat */
        u64 r = 1, a = d->n % q, e = q - 2;
        while (e) { if (e & 1) r = mm(r, a, q); a = mm(a, a, q); e >>= 1; }
        d->ninv[p] = r;
        d->ninvS[p] = (u64)(((u128)r << 64) / q);
    }
    return d;
}

void sfp_destroy(sfp_dev* d) {
    if (!d) return;
    free(d->q); free(d->psi); free(d->ipsi); free(d->psiS); free(d->ipsiS);
    free(d->ninv); free(d->ninvS);
    free(d->enc_rot); free(d->enc_ksi);
    free(d);
}

void* sfp_alloc(sfp_dev* d, size_t bytes) { (void)d; return malloc(bytes ? bytes : 8); }
void sfp_free(sfp_dev* d, void* p) { (void)d; free(p); }
void sfp_h2d(sfp_dev* d, void* dst, const void* src, size_t b) { (void)d; memcpy(dst, src, b); }
void sfp_d2h(sfp_dev* d, void* dst, const void* src, size_t b) { (void)d; memcpy(dst, src, b); }
void sfp_d2d(sfp_dev* d, void* dst, const void* src, size_t b) { (void)d; memmove(dst, src, b); }
void sfp_zero(sfp_dev* d, void* dst, size_t b) { (void)d; memset(dst, 0, b); }
void sfp_sync(sfp_dev* d) { (void)d; }
/* one synchronous lane: everything is already ordered */
struct sfp_event { int lane; };
static struct sfp_event g_oracle_event = {0};
int sfp_lanes(sfp_dev* d) { (void)d; return 8; }
void sfp_set_lane(sfp_dev* d, int lane) { (void)d; (void)lane; }
int sfp_get_lane(sfp_dev* d) { (void)d; return 0; }
sfp_event* sfp_event_record(sfp_dev* d) { (void)d; return &g_oracle_event; }
void sfp_event_wait(sfp_dev* d, const sfp_event* e) { (void)d; (void)e; }
int sfp_event_done(sfp_dev* d, const sfp_event* e) { (void)d; (void)e; return 1; }
void sfp_event_free(sfp_dev* d, sfp_event* e) { (void)d; (void)e; }
void sfp_lane_wait(sfp_dev* d, int waiter, int waitee) { (void)d; (void)waiter; (void)waitee; }
/* kernel timing is a device-backend feature; the oracle reports nothing */
void sfp_prof_set(sfp_dev* d, uint32_t fam, uint32_t period) { (void)d; (void)fam; (void)period; }
int sfp_graph_family_time(sfp_dev* d, sfp_graph* g, uint32_t fam, int reps, double* ms, uint64_t* launches,
                          double* bytes) {
    (void)d; (void)g; (void)fam; (void)reps; (void)ms; (void)launches; (void)bytes;
    return -1;
}
void sfp_serialize(sfp_dev* d, int on) { (void)d; (void)on; }
/* one synchronous lane: nothing to stack */
void sfp_stack_begin(sfp_dev* d) { (void)d; }
void sfp_stack_end(sfp_dev* d) { (void)d; }
int sfp_batch_begin(sfp_dev* d, uint32_t count) {
    (void)d;
    (void)count;
    return 0;
}
void sfp_batch_lane(sfp_dev* d, uint32_t i) { (void)d; (void)i; }
void sfp_batch_end(sfp_dev* d) { (void)d; }
void sfp_stack_stats(sfp_dev* d, uint64_t* merged, uint64_t* single) {
    (void)d;
    if (merged) *merged = 0;
    if (single) *single = 0;
}
/* no graphs: the host layer runs every region eagerly */
int sfp_capture_begin(sfp_dev* d) { (void)d; return -1; }
void sfp_clear_error(sfp_dev* d) { (void)d; }
sfp_graph* sfp_capture_end(sfp_dev* d) { (void)d; return NULL; }
int sfp_capturing(sfp_dev* d) { (void)d; return 0; }
void sfp_graph_launch(sfp_dev* d, sfp_graph* g) { (void)d; (void)g; }
size_t sfp_graph_nodes(const sfp_graph* g) { (void)g; return 0; }
void sfp_graph_destroy(sfp_dev* d, sfp_graph* g) { (void)d; (void)g; }
int sfp_prof_read(sfp_dev* d, uint32_t fam, uint64_t* launches, uint64_t* timed, double* ms,
                  double* bytes) {
    (void)d; (void)fam;
    if (launches) *launches = 0;
    if (timed) *timed = 0;
    if (ms) *ms = 0;
    if (bytes) *bytes = 0;
    return 0;
}
const char* sfp_last_error(sfp_dev* d) { (void)d; return NULL; }

/* ---- NTT ---- */
static void ntt_fwd(const sfp_dev* d, u64* a, uint32_t p) {
    const uint32_t n = d->n;
    const u64 q = d->q[p];
    const u64* w = d->psi + (size_t)p * n;
    const u64* wp = d->psiS + (size_t)p * n;
    uint32_t t = n;
    for (uint32_t m = 1; m < n; m <<= 1) {
        t >>= 1;
        for (uint32_t i = 0; i < m; ++i) {
            uint32_t j1 = 2 * i * t;
            u64 S = w[m + i], Sp = wp[m + i];
            for (uint32_t j = j1; j < j1 + t; ++j) {
                u64 U = a[j], V = shoup(a[j + t], S, Sp, q);
                a[j] = ad(U, V, q);
                a[j + t] = sb(U, V, q);
            }
        }
    }
}
static void ntt_inv(const sfp_dev* d, u64* a, uint32_t p) {
    const uint32_t n = d->n;
    const u64 q = d->q[p];
    const u64* w = d->ipsi + (size_t)p * n;
    const u64* wp = d->ipsiS + (size_t)p * n;
    uint32_t t = 1;
    for (uint32_t m = n; m > 1; m >>= 1) {
        uint32_t j1 = 0, h = m >> 1;
        for (uint32_t i = 0; i < h; ++i) {
            u64 S = w[h + i], Sp = wp[h + i];
            for (uint32_t j = j1; j < j1 + t; ++j) {
                u64 U = a[j], V = a[j + t];
                a[j] = ad(U, V, q);
                a[j + t] = shoup(sb(U, V, q), S, Sp, q);
            }
            j1 += 2 * t;
        }
        t <<= 1;
    }
    for (uint32_t j = 0; j < n; ++j) a[j] = shoup(a[j], d->ninv[p], d->ninvS[p], q);
}

void sfp_ntt_batch(sfp_dev* d, uint64_t* p, size_t stride, uint32_t count, sfp_limbs m, int inverse) {
    for (uint32_t b = 0; b < count; ++b) sfp_ntt(d, p + (size_t)b * stride, m, inverse);
}

void sfp_ntt(sfp_dev* d, uint64_t* p, sfp_limbs m, int inverse) {
#pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < m.count; ++i) {
        if (inverse) ntt_inv(d, p + (size_t)i * d->n, pidx(m, i));
        else ntt_fwd(d, p + (size_t)i * d->n, pidx(m, i));
    }
}

/* ---- elementwise ---- */
#define LOOP_LIMBS(...)                                                \
    _Pragma("omp parallel for schedule(static)")                       \
    for (uint32_t i = 0; i < m.count; ++i) {                            \
        const u64 q = d->q[pidx(m, i)];                                 \
        const size_t o = (size_t)i * d->n;                              \
        (void)q;                                                        \
        for (uint32_t x = 0; x < d->n; ++x) { __VA_ARGS__; }            \
    }

void sfp_add(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m) {
    LOOP_LIMBS(out[o + x] = ad(a[o + x], b[o + x], q))
}
void sfp_sub(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m) {
    LOOP_LIMBS(out[o + x] = sb(a[o + x], b[o + x], q))
}
void sfp_neg(sfp_dev* d, uint64_t* out, const uint64_t* a, sfp_limbs m) {
    LOOP_LIMBS(out[o + x] = a[o + x] ? q - a[o + x] : 0)
}
void sfp_mul(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m) {
    LOOP_LIMBS(out[o + x] = mm(a[o + x], b[o + x], q))
}
void sfp_mul_add(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b,
                 const uint64_t* c, sfp_limbs m) {
    LOOP_LIMBS(out[o + x] = ad(mm(a[o + x], b[o + x], q), c[o + x], q))
}
void sfp_mul_const(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* k, sfp_limbs m) {
    LOOP_LIMBS(out[o + x] = mm(a[o + x], k[i], q))
}
void sfp_add_const(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* k, sfp_limbs m) {
    LOOP_LIMBS(out[o + x] = ad(a[o + x], k[i], q))
}
void sfp_tensor(sfp_dev* d, uint64_t* d0, uint64_t* d1, uint64_t* d2, const uint64_t* a0,
                const uint64_t* a1, const uint64_t* b0, const uint64_t* b1, sfp_limbs m) {
    LOOP_LIMBS({
        u64 x0 = a0[o + x], x1 = a1[o + x], y0 = b0[o + x], y1 = b1[o + x];
        u64 r0 = mm(x0, y0, q), r1 = ad(mm(x0, y1, q), mm(x1, y0, q), q), r2 = mm(x1, y1, q);
        d0[o + x] = r0; d1[o + x] = r1; d2[o + x] = r2;
    })
}
void sfp_lin_wsum(sfp_dev* d, uint64_t* out, const uint64_t* const* ins, const uint64_t* k,
                  uint32_t nin, sfp_limbs m) {
    LOOP_LIMBS({
        u128 acc = 0;
        for (uint32_t j = 0; j < nin; ++j) acc += (u128)ins[j][o + x] * k[(size_t)j * m.count + i];
        out[o + x] = (u64)(acc % q);
    })
}

void sfp_mac_plain2(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* const* a0,
                    const uint64_t* const* a1, const uint64_t* const* b, uint32_t nin, sfp_limbs m) {
    sfp_mac_plain(d, out0, a0, b, nin, m);
    sfp_mac_plain(d, out1, a1, b, nin, m);
}

/* the multi-output form: ng separate sums, exactly as ng sfp_mac_plain2 calls */
int sfp_mac_plain2_multi(sfp_dev* d, uint64_t* const* out0, uint64_t* const* out1, const uint64_t* const* a0,
                         const uint64_t* const* a1, const uint64_t* const* b, uint32_t nin, uint32_t ng,
                         sfp_limbs m) {
    if (!ng || ng > SFP_MAC_MULTI_G || !nin || nin > SFP_MAC_MULTI_N) return -1;
    for (uint32_t g = 0; g < ng; ++g) sfp_mac_plain2(d, out0[g], out1[g], a0, a1, b + (size_t)g * nin, nin, m);
    return 0;
}

void sfp_mac_plain(sfp_dev* d, uint64_t* out, const uint64_t* const* a, const uint64_t* const* b,
                   uint32_t nin, sfp_limbs m) {
    LOOP_LIMBS({
        u128 acc = 0;
        for (uint32_t j = 0; j < nin; ++j) acc += (u128)a[j][o + x] * b[j][o + x];
        out[o + x] = (u64)(acc % q);
    })
}

/* ---- automorphism ---- */
void sfp_automorph(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t g, sfp_limbs m) {
    const uint32_t n = d->n, logn = d->logn;
    const u64 twoN = 2ull * n;
    uint32_t* perm = (uint32_t*)malloc(n * 4);
    for (uint32_t k = 0; k < n; ++k) {
        u64 e = 2ull * brev(k, logn) + 1;
        u64 ge = (e * g) % twoN;
        perm[k] = brev((uint32_t)((ge - 1) / 2), logn);
    }
#pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < m.count; ++i) {
        const size_t o = (size_t)i * n;
        for (uint32_t k = 0; k < n; ++k) out[o + k] = in[o + perm[k]];
    }
    free(perm);
}

void sfp_lin_wsum_multi(sfp_dev* d, uint64_t* out, size_t out_stride, size_t poly_stride,
                        const uint64_t* const* in0, const uint64_t* const* in1, uint32_t nin,
                        const uint64_t* k, uint32_t nout, sfp_limbs m) {
    const uint64_t** ins = (const uint64_t**)malloc(nin * sizeof(uint64_t*));
    uint64_t* kk = (uint64_t*)malloc((size_t)nin * m.count * 8);
    for (uint32_t o = 0; o < nout; ++o) {
        memcpy(kk, k + (size_t)o * nin * m.count, (size_t)nin * m.count * 8);
        for (int p = 0; p < 2; ++p) {
            for (uint32_t j = 0; j < nin; ++j) ins[j] = p ? in1[j] : in0[j];
            sfp_lin_wsum(d, out + o * out_stride + p * poly_stride, ins, kk, nin, m);
        }
    }
    free(ins);
    free(kk);
}

/* ---- rescale ---- */
void sfp_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t ell, const uint64_t* qlinv,
                 uint32_t npoly, size_t in_stride, size_t out_stride) {
    sfp_rescale_ext(d, out, in, ell, ell - 1, qlinv, npoly, in_stride, out_stride);
}

void sfp_rescale_ext(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t ell, uint32_t drop_prime,
                     const uint64_t* qlinv, uint32_t npoly, size_t in_stride, size_t out_stride) {
    const uint32_t n = d->n;
    const u64 ql = d->q[drop_prime];
    u64* last = (u64*)malloc((size_t)n * 8);
    for (uint32_t p = 0; p < npoly; ++p) {
        const u64* src = in + p * in_stride;
        u64* dst = out + p * out_stride;
        memcpy(last, src + (size_t)(ell - 1) * n, (size_t)n * 8);
        ntt_inv(d, last, drop_prime);
#pragma omp parallel for schedule(static)
        for (uint32_t i = 0; i < ell - 1; ++i) {
            const u64 q = d->q[i];
            u64* row = (u64*)malloc((size_t)n * 8);
            const u64 qlmod = ql % q;
            for (uint32_t x = 0; x < n; ++x) {
                u64 v = last[x];
                u64 r = v % q;
                if (v > (ql >> 1)) r = sb(r, qlmod, q); /* centred: v - q_l */
                row[x] = r;
            }
            ntt_fwd(d, row, i);
            const size_t o = (size_t)i * n;
            for (uint32_t x = 0; x < n; ++x) dst[o + x] = mm(sb(src[o + x], row[x], q), qlinv[i], q);
            free(row);
        }
    }
    free(last);
}

/* fused product + rescale (prims.h), stated as the two steps */
void sfp_mul_const_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* k,
                           uint32_t ell, const uint64_t* qlinv, uint32_t npoly, size_t in_stride,
                           size_t out_stride) {
    const size_t w = (size_t)ell * d->n;
    u64* t = (u64*)malloc(w * npoly * 8);
    for (uint32_t p = 0; p < npoly; ++p)
        sfp_mul_const(d, t + p * w, in + p * in_stride, k, (sfp_limbs){ell, ell, 0, 0});
    sfp_rescale(d, out, t, ell, qlinv, npoly, w, out_stride);
    free(t);
}
void sfp_mul_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* m, uint32_t ell,
                     const uint64_t* qlinv, uint32_t npoly, size_t in_stride, size_t out_stride) {
    const size_t w = (size_t)ell * d->n;
    u64* t = (u64*)malloc(w * npoly * 8);
    for (uint32_t p = 0; p < npoly; ++p)
        sfp_mul(d, t + p * w, in + p * in_stride, m, (sfp_limbs){ell, ell, 0, 0});
    sfp_rescale(d, out, t, ell, qlinv, npoly, w, out_stride);
    free(t);
}

/* ---- base conversion / key switching ---- */
sfp_conv* sfp_upload_conv(sfp_dev* d, uint32_t ns, const uint32_t* src, uint32_t nt,
                          const uint32_t* dst, const uint32_t* drow, const uint64_t* inv,
                          const uint64_t* mod) {
    sfp_conv* c = (sfp_conv*)calloc(1, sizeof(sfp_conv));
    c->ns = ns; c->nt = nt;
    c->drow = (uint32_t*)malloc(nt * 4);
    for (uint32_t t = 0; t < nt; ++t) c->drow[t] = drow ? drow[t] : t;
    c->src = (uint32_t*)malloc(ns * 4); memcpy(c->src, src, ns * 4);
    c->dst = (uint32_t*)malloc(nt * 4); memcpy(c->dst, dst, nt * 4);
    c->inv = (u64*)malloc(ns * 8); memcpy(c->inv, inv, ns * 8);
    c->mod = (u64*)malloc((size_t)ns * nt * 8); memcpy(c->mod, mod, (size_t)ns * nt * 8);
    c->sprod = (u64*)malloc(nt * 8);
    for (uint32_t t = 0; t < nt; ++t) {
        u64 pt = d->q[dst[t]], r = 1;
        for (uint32_t i = 0; i < ns; ++i) r = mm(r, d->q[src[i]] % pt, pt);
        c->sprod[t] = r;
    }
    return c;
}
void sfp_free_conv(sfp_dev* d, sfp_conv* c) {
    (void)d;
    if (!c) return;
    free(c->src); free(c->dst); free(c->inv); free(c->mod); free(c->sprod); free(c->drow); free(c);
}

/* dst row t (prime c->dst[t]) = sum_i [src_i * inv_i]_{s_i} * mod[i][t]  (coefficient domain).
 * centered: the EXACT centred conversion (ModDown).  Each y_i is taken in
 * (-s_i/2, s_i/2], and the overflow v = round(sum_i y_i / s_i) is removed:
 *   out_t = sum_i y_i * mod[i][t] - v * prod(S)   (mod t),
 * which is the centred representative of x mod prod(S) itself, so ModDown's
 * division by P leaves only its rounding (|x / P| <= 1/2) instead of the fast
 * conversion's integer overflow v (variance ~K/12: ~sqrt(K+1) x the noise).
 * v is estimated in FP64 exactly as the HIP kernels do it (same operations,
 * same order): acc = fma((double)y_i, 1.0 / (double)s_i, acc), v = rint(acc). */
static void conv_rows(const sfp_dev* d, const sfp_conv* c, const u64* src, u64* const* dstRows,
                      uint32_t ntUse, int centered) {
    const uint32_t n = d->n;
#pragma omp parallel for schedule(static)
    for (uint32_t x = 0; x < n; ++x) {
        u64 y[SFP_MAX_LIMBS];
        int64_t m = 0; /* multiples of prod(S) to subtract: one per negative y_i, plus v */
        double acc = 0.0;
        for (uint32_t i = 0; i < c->ns; ++i) {
            u64 qi = d->q[c->src[i]];
            y[i] = mm(src[(size_t)i * n + x], c->inv[i], qi);
            if (centered) {
                int64_t yc = (int64_t)y[i];
                if (y[i] > (qi >> 1)) {
                    ++m;
                    yc -= (int64_t)qi;
                }
                acc = fma((double)yc, 1.0 / (double)qi, acc);
            }
        }
        if (centered) m += (int64_t)rint(acc);
        for (uint32_t t = 0; t < ntUse; ++t) {
            u64 pt = d->q[c->dst[t]];
            u128 a = 0;
            for (uint32_t i = 0; i < c->ns; ++i) a += (u128)y[i] * c->mod[(size_t)i * c->nt + t];
            u64 v = (u64)(a % pt);
            if (m > 0) v = sb(v, mm((u64)m, c->sprod[t], pt), pt);
            if (m < 0) v = ad(v, mm((u64)(-m), c->sprod[t], pt), pt);
            dstRows[t][x] = v;
        }
    }
}

void sfp_conv_apply(sfp_dev* d, uint64_t* dst, const uint64_t* src, const sfp_conv* c) {
    u64** rows = (u64**)malloc(c->nt * sizeof(u64*));
    for (uint32_t t = 0; t < c->nt; ++t) rows[t] = dst + (size_t)c->drow[t] * d->n;
    conv_rows(d, c, src, rows, c->nt, 0);
    free(rows);
}

/* centred conversion onto the first nt_use targets (the sharded ModDown's P -> local Q) */
void sfp_conv_apply_centered(sfp_dev* d, uint64_t* dst, const uint64_t* src, const sfp_conv* c,
                             uint32_t nt_use) {
    if (!c || !nt_use) return;
    u64** rows = (u64**)malloc(nt_use * sizeof(u64*));
    for (uint32_t t = 0; t < nt_use; ++t) rows[t] = dst + (size_t)c->drow[t] * d->n;
    conv_rows(d, c, src, rows, nt_use, 1);
    free(rows);
}

/* every digit j: own rows copied, the others NTT(Conv_j(INTT(in[digit j]))) */
void sfp_modup(sfp_dev* d, uint64_t* ext, const uint64_t* in, uint32_t ell, uint32_t K,
               uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, uint64_t* scratch) {
    const uint32_t n = d->n;
    const uint32_t beta = (ell + alpha - 1) / alpha;
    const size_t stride = (size_t)(ell + K) * n;
    (void)Lq;
    memcpy(scratch, in, (size_t)ell * n * 8);
#pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < ell; ++i) ntt_inv(d, scratch + (size_t)i * n, i);
    for (uint32_t j = 0; j < beta; ++j) {
        const sfp_conv* c = convs[j];
        const uint32_t lo = j * alpha, hi = lo + alpha < ell ? lo + alpha : ell;
        u64* out = ext + j * stride;
        u64** rows = (u64**)malloc(c->nt * sizeof(u64*));
        for (uint32_t t = 0; t < c->nt; ++t) rows[t] = out + (size_t)c->drow[t] * n;
        conv_rows(d, c, scratch + (size_t)lo * n, rows, c->nt, 0);
#pragma omp parallel for schedule(static)
        for (uint32_t t = 0; t < c->nt; ++t) ntt_fwd(d, rows[t], c->dst[t]);
        free(rows);
        memcpy(out + (size_t)lo * n, in + (size_t)lo * n, (size_t)(hi - lo) * n * 8);
    }
}

void sfp_ks_inner(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                  size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                  uint32_t Lq) {
    sfp_ks_inner_fold(d, acc0, acc1, ext, ext_stride, key, beta, ell, K, Lq, NULL, NULL, 0);
}

static void ks_inner_rows(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                          size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell,
                          uint32_t K, uint32_t Lq, const uint64_t* fold0, const uint64_t* fold1,
                          uint64_t fold_k, int accum, const uint64_t* pm);

void sfp_ks_inner_mul(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                      size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                      uint32_t Lq, const uint64_t* pm, int accum) {
    ks_inner_rows(d, acc0, acc1, ext, ext_stride, key, beta, ell, K, Lq, NULL, NULL, 0, accum, pm);
}

void sfp_ks_inner_fold(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                       size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell,
                       uint32_t K, uint32_t Lq, const uint64_t* fold0, const uint64_t* fold1,
                       uint64_t fold_k) {
    ks_inner_rows(d, acc0, acc1, ext, ext_stride, key, beta, ell, K, Lq, fold0, fold1, fold_k, 0, NULL);
}

void sfp_ks_inner_acc(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                      size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                      uint32_t Lq) {
    ks_inner_rows(d, acc0, acc1, ext, ext_stride, key, beta, ell, K, Lq, NULL, NULL, 0, 1, NULL);
}

/* the digits permuted by X -> X^gal (sfp_automorph), then sfp_ks_inner_mul */
void sfp_ks_inner_mul_aut(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                          size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                          uint32_t Lq, const uint64_t* pm, int accum, uint32_t gal) {
    const uint32_t rows = (uint32_t)(ext_stride / d->n);
    uint64_t* t = (uint64_t*)malloc(ext_stride * beta * 8);
    sfp_limbs m;
    memset(&m, 0, sizeof m);
    m.count = rows;
    m.split = rows;
    for (uint32_t j = 0; j < beta; ++j) sfp_automorph(d, t + j * ext_stride, ext + j * ext_stride, gal, m);
    sfp_ks_inner_mul(d, acc0, acc1, t, ext_stride, key, beta, ell, K, Lq, pm, accum);
    free(t);
}

/* the digits permuted by X -> X^gal (sfp_automorph), then sfp_ks_inner */
void sfp_ks_inner_aut(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                      size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                      uint32_t Lq, uint32_t gal) {
    const uint32_t rows = (uint32_t)(ext_stride / d->n);
    uint64_t* t = (uint64_t*)malloc(ext_stride * beta * 8);
    sfp_limbs m;
    memset(&m, 0, sizeof m);
    m.count = rows;
    m.split = rows;
    for (uint32_t j = 0; j < beta; ++j) sfp_automorph(d, t + j * ext_stride, ext + j * ext_stride, gal, m);
    sfp_ks_inner(d, acc0, acc1, t, ext_stride, key, beta, ell, K, Lq);
    free(t);
}

// acc (+)= sum_j ext_j * key_j (mod q) per ext limb (sfp_ks_inner / _fold / _acc)
static void ks_inner_rows(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                          size_t ext_stride, const uint64_t* key, uint32_t beta, uint32_t ell,
                          uint32_t K, uint32_t Lq, const uint64_t* fold0, const uint64_t* fold1,
                          uint64_t fold_k, int accum, const uint64_t* pm) {
    const uint32_t n = d->n, rows = ell + K, NP = d->kg.rows ? d->kg.rows : Lq + K;
    const uint32_t pst = d->kg.rows ? d->kg.pstart : Lq;
#pragma omp parallel for schedule(static)
    for (uint32_t t = 0; t < rows; ++t) {
        const uint32_t kr = t < ell ? t : pst + (t - ell);  /* key row */
        const u64 q = d->q[t < ell ? t : Lq + (t - ell)];
        for (uint32_t x = 0; x < n; ++x) {
            u128 s0 = 0, s1 = 0;
            for (uint32_t j = 0; j < beta; ++j) {
                u64 e = ext[j * ext_stride + (size_t)t * n + x];
                const u64* kb = key + (size_t)j * 2 * NP * n;
                const u64* ka = kb + (size_t)NP * n;
                s0 += (u128)e * kb[(size_t)kr * n + x];
                s1 += (u128)e * ka[(size_t)kr * n + x];
            }
            if (fold0 && t == ell - 1) {
                s0 += (u128)fold0[(size_t)t * n + x] * fold_k;
                s1 += (u128)fold1[(size_t)t * n + x] * fold_k;
            }
            if (pm) {  /* (sum mod q) * pm mod q */
                const u64 m = pm[(size_t)t * n + x];
                s0 = (u128)(u64)(s0 % q) * m;
                s1 = (u128)(u64)(s1 % q) * m;
            }
            if (accum) {
                s0 = (u128)(u64)(s0 % q) + acc0[(size_t)t * n + x];
                s1 = (u128)(u64)(s1 % q) + acc1[(size_t)t * n + x];
            }
            acc0[(size_t)t * n + x] = (u64)(s0 % q);
            acc1[(size_t)t * n + x] = (u64)(s1 % q);
        }
    }
}

static void moddown1(sfp_dev* d, uint64_t* out, uint64_t* acc, uint32_t ell, uint32_t K,
                     uint32_t Lq, const sfp_conv* c, const uint64_t* pinv, int add,
                     uint64_t* scratch) {
    const uint32_t n = d->n;
    u64* pRows = acc + (size_t)ell * n;
    for (uint32_t k = 0; k < K; ++k) ntt_inv(d, pRows + (size_t)k * n, Lq + k);
    u64** rows = (u64**)malloc(ell * sizeof(u64*));
    for (uint32_t i = 0; i < ell; ++i) rows[i] = scratch + (size_t)i * n;
    conv_rows(d, c, pRows, rows, ell, 1);
#pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < ell; ++i) {
        const u64 q = d->q[i];
        ntt_fwd(d, rows[i], i);
        const size_t o = (size_t)i * n;
        for (uint32_t x = 0; x < n; ++x) {
            u64 v = mm(sb(acc[o + x], rows[i][x], q), pinv[i], q);
            out[o + x] = add ? ad(out[o + x], v, q) : v;
        }
    }
    free(rows);
}

void sfp_moddown2(sfp_dev* d, uint64_t* out0, uint64_t* out1, uint64_t* acc, size_t acc_stride,
                  uint32_t ell, uint32_t K, uint32_t Lq, const sfp_conv* c, const uint64_t* pinv,
                  int add0, int add1, uint64_t* scratch, int row_done) {
    (void)row_done; /* never set: the oracle has no sfp_modup_inner */
    moddown1(d, out0, acc, ell, K, Lq, c, pinv, add0, scratch);
    moddown1(d, out1, acc + acc_stride, ell, K, Lq, c, pinv, add1, scratch + (size_t)ell * d->n);
}

/* ModDown + add + rescale, stated as the two steps it fuses (prims.h):
 * ModDown of the folded accumulators, add d on rows < l (row l already holds
 * P d_l through the fold), then Rescale. */
void sfp_moddown_rescale(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* d0,
                         const uint64_t* d1, uint64_t* acc, size_t acc_stride, uint32_t ell,
                         uint32_t K, uint32_t Lq, const sfp_conv* c, const uint64_t* pinv,
                         const uint64_t* pmod, const uint64_t* qlinv, uint64_t* scratch, int row_done) {
    const uint32_t n = d->n, l = ell - 1;
    (void)pmod;
    (void)row_done; /* never set: the oracle has no sfp_modup_inner */
    u64* s = (u64*)malloc((size_t)ell * n * 8);
    for (int p = 0; p < 2; ++p) {
        const u64* dp = p ? d1 : d0;
        u64* op = p ? out1 : out0;
        moddown1(d, s, acc + (size_t)p * acc_stride, ell, K, Lq, c, pinv, 0, scratch);
        for (uint32_t i = 0; i < l; ++i) {
            const u64 q = d->q[i];
            for (uint32_t x = 0; x < n; ++x) s[(size_t)i * n + x] = ad(s[(size_t)i * n + x], dp[(size_t)i * n + x], q);
        }
        sfp_rescale(d, op, s, ell, qlinv, 1, 0, 0);
    }
    free(s);
}

/* ---- sampling / loading ---- */
static inline u64 smix(u64 x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
void sfp_sample_uniform(sfp_dev* d, uint64_t* p, sfp_limbs m, uint64_t seed) {
#pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < m.count; ++i) {
        const uint32_t pi = pidx(m, i);
        const u64 q = d->q[pi];
        const u64 base = smix(seed ^ (0xD1B54A32D192ED03ULL * (u64)(pi + 1)));
        for (uint32_t x = 0; x < d->n; ++x) {
            u64 r0 = smix(base + 2ull * x), r1 = smix(base + 2ull * x + 1);
            p[(size_t)i * d->n + x] = (u64)((((u128)r1 << 64) | r0) % q);
        }
    }
}
void sfp_load_i64(sfp_dev* d, uint64_t* p, const int64_t* c, sfp_limbs m) {
    LOOP_LIMBS({
        int64_t v = c[x];
        u64 a = v < 0 ? (u64)(-(v + 1)) + 1 : (u64)v;
        u64 r = a % q;
        p[o + x] = (v < 0 && r) ? q - r : r;
    })
}

/* no fused ModUp + inner product: the host layer runs sfp_modup + sfp_ks_inner* */
int sfp_modup_inner(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* in, uint32_t ell, uint32_t K,
                    uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key,
                    const uint64_t* fold0, const uint64_t* fold1, uint64_t fold_k, int accum, uint32_t inv_from,
                    uint64_t* ext, uint64_t* scratch) {
    (void)d; (void)acc0; (void)acc1; (void)in; (void)ell; (void)K; (void)Lq; (void)alpha; (void)convs;
    (void)key; (void)fold0; (void)fold1; (void)fold_k; (void)accum; (void)inv_from; (void)ext; (void)scratch;
    return -1;
}
int sfp_modup_inner_phase(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* in, uint32_t ell, uint32_t K,
                          uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key,
                          const uint64_t* fold0, const uint64_t* fold1, uint64_t fold_k, int accum,
                          uint32_t inv_from, uint64_t* ext, uint64_t* scratch, int phases) {
    (void)phases; /* no fused form: the caller runs the unfused prims */
    return sfp_modup_inner(d, acc0, acc1, in, ell, K, Lq, alpha, convs, key, fold0, fold1, fold_k, accum, inv_from,
                           ext, scratch);
}

/* no fused ModUp: nothing to prepare */
void sfp_modup_prepare(sfp_dev* d, const sfp_conv* const* convs, uint32_t ell, uint32_t K, uint32_t alpha) {
    (void)d; (void)convs; (void)ell; (void)K; (void)alpha;
}

/* no fused tensor + relinearisation + rescale: the host layer runs the prims */
int sfp_mult_relin_rescale(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* a0, const uint64_t* a1,
                           const uint64_t* b0, const uint64_t* b1, uint32_t ell, uint32_t K, uint32_t Lq,
                           uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key, const sfp_conv* c,
                           const uint64_t* pinv, const uint64_t* pmod, const uint64_t* qlinv, uint64_t* acc,
                           uint64_t* ext, uint64_t* scratch) {
    (void)d; (void)out0; (void)out1; (void)a0; (void)a1; (void)b0; (void)b1; (void)ell; (void)K; (void)Lq;
    (void)alpha; (void)convs; (void)key; (void)c; (void)pinv; (void)pmod; (void)qlinv; (void)acc; (void)ext;
    (void)scratch;
    return -1;
}

/* ---- CKKS encoding (sfp_encode): the host encoder's special inverse FFT
 * (csrc/core/encoder.cpp fftSpecialInv) restated in C, then round and reduce
 * as sfp_load_i64.  Built with -ffp-contract=off: no fused multiply-add. */
void sfp_encode_setup(sfp_dev* d, const uint64_t* rot, const double* ksi) {
    free(d->enc_rot);
    free(d->enc_ksi);
    d->enc_rot = (u64*)malloc((size_t)d->n / 2 * 8);
    d->enc_ksi = (double*)malloc((size_t)(2 * d->n + 1) * 16);
    memcpy(d->enc_rot, rot, (size_t)d->n / 2 * 8);
    memcpy(d->enc_ksi, ksi, (size_t)(2 * d->n + 1) * 16);
}

void sfp_encode(sfp_dev* d, uint64_t* p, const double* vals, uint32_t nvals, int real, uint32_t slots,
                double scale, sfp_limbs m, uint64_t* scratch);
void sfp_encode_batch(sfp_dev* d, uint64_t* dst, size_t dstStride, const double* vals, uint32_t nvals,
                      uint32_t count, int real, uint32_t slots, double scale, sfp_limbs m, uint64_t* scratch) {
    for (uint32_t b = 0; b < count; ++b)
        sfp_encode(d, dst + (size_t)b * dstStride, vals + (size_t)b * nvals * (real ? 1 : 2), nvals, real, slots,
                   scale, m, scratch);
}

void sfp_encode(sfp_dev* d, uint64_t* p, const double* vals, uint32_t nvals, int real, uint32_t slots,
                double scale, sfp_limbs m, uint64_t* scratch) {
    const uint32_t n = d->n, S = slots;
    const u64 M = 2ull * n;
    double* v = (double*)scratch; /* S (re, im) pairs */
    for (uint32_t i = 0; i < S; ++i) {
        v[2 * i] = i < nvals ? (real ? vals[i] : vals[2 * i]) : 0.0;
        v[2 * i + 1] = i < nvals && !real ? vals[2 * i + 1] : 0.0;
    }
    for (uint32_t len = S; len >= 1; len >>= 1) {
        const uint32_t lenh = len >> 1;
        const u64 lenq = (u64)len << 2;
        for (uint32_t i = 0; i < S; i += len)
            for (uint32_t j = 0; j < lenh; ++j) {
                const u64 idx = (lenq - (d->enc_rot[j] % lenq)) * M / lenq;
                double* a = v + 2 * (size_t)(i + j);
                double* b = v + 2 * (size_t)(i + j + lenh);
                const double kr = d->enc_ksi[2 * idx], ki = d->enc_ksi[2 * idx + 1];
                const double ur = a[0] + b[0], ui = a[1] + b[1];
                const double dr = a[0] - b[0], di = a[1] - b[1];
                a[0] = ur;
                a[1] = ui;
                b[0] = dr * kr - di * ki;
                b[1] = dr * ki + di * kr;
            }
        if (len == 1) break;
    }
    uint32_t logS = 0;
    while ((1u << logS) < S) ++logS;
    const uint32_t half = n / 2, gap = half / S;
    LOOP_LIMBS({
        const uint32_t xi = x < half ? x : x - half;
        int64_t c = 0;
        if (xi % gap == 0) {
            const uint32_t i = xi / gap;
            uint32_t r = 0;
            for (uint32_t b = 0; b < logS; ++b) r |= ((i >> b) & 1u) << (logS - 1 - b);
            const double u = v[2 * (size_t)r + (x < half ? 0 : 1)] / (double)S;
            c = (int64_t)nearbyint(u * scale);
        }
        u64 a = c < 0 ? (u64)(-(c + 1)) + 1 : (u64)c;
        u64 rr = a % q;
        p[o + x] = (c < 0 && rr) ? q - rr : rr;
    })
}

/* ---- limb sharding ---- */
int sfp_comm_uid(void* uid128) { (void)uid128; return -1; }
int sfp_comm_init_rccl(sfp_dev* d, int rank, int world, const void* uid128) {
    (void)d; (void)rank; (void)world; (void)uid128;
    return -1; /* no RCCL in the oracle: host callbacks only */
}
void sfp_comm_set_host(sfp_dev* d, int rank, int world, sfp_host_allgather_fn ag, sfp_host_bcast_fn bc,
                       void* user) {
    d->rank = rank;
    d->world = world;
    d->ag = ag;
    d->bc = bc;
    d->user = user;
}
int sfp_comm_capturable(sfp_dev* d) { (void)d; return 0; /* no graphs in the oracle */ }
static double comm_now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}
void sfp_comm_stats_reset(sfp_dev* d, int timed) {
    d->comm_calls = 0;
    d->comm_bytes = 0;
    d->comm_ms = 0;
    d->comm_timed = timed;
}
void sfp_comm_stats(sfp_dev* d, uint64_t* calls, double* bytes, double* ms) {
    if (calls) *calls = d->comm_calls;
    if (bytes) *bytes = d->comm_bytes;
    if (ms) *ms = d->comm_ms;
}
/* one host collective: counted, and timed by the wall clock (the oracle is synchronous) */
static double comm_begin(sfp_dev* d) { return d->comm_timed ? comm_now_ms() : 0.0; }
static void comm_end(sfp_dev* d, double t0, double received) {
    d->comm_calls++;
    d->comm_bytes += received;
    if (d->comm_timed) d->comm_ms += comm_now_ms() - t0;
}
void sfp_allgather(sfp_dev* d, const void* send, void* recv, size_t bytes) {
    if (d->world <= 1 || !d->ag) {
        if (send != recv) memmove(recv, send, bytes);
        return;
    }
    const double t0 = comm_begin(d);
    void* tmp = malloc(bytes ? bytes : 1); /* send may alias recv */
    memcpy(tmp, send, bytes);
    d->ag(d->user, tmp, recv, bytes);
    free(tmp);
    comm_end(d, t0, (double)bytes * (d->world - 1));
}
int sfp_group_init_rccl(sfp_dev* d, int group, int groups, const void* uid128) {
    (void)d; (void)group; (void)groups; (void)uid128;
    return -1; /* no RCCL in the oracle */
}
void sfp_group_set_host(sfp_dev* d, int group, int groups, sfp_host_allgather_fn ag, void* user) {
    d->grank = group;
    d->gworld = groups;
    d->gag = ag;
    d->guser = user;
}
void sfp_group_allgather(sfp_dev* d, const void* send, void* recv, size_t bytes) {
    if (d->gworld <= 1 || !d->gag) {
        if (send != recv) memmove(recv, send, bytes);
        return;
    }
    const double t0 = comm_begin(d);
    void* tmp = malloc(bytes ? bytes : 1);
    memcpy(tmp, send, bytes);
    d->gag(d->guser, tmp, recv, bytes);
    free(tmp);
    comm_end(d, t0, (double)bytes * (d->gworld - 1));
}
void sfp_bcast(sfp_dev* d, void* buf, size_t bytes, int root) {
    if (d->world <= 1 || !d->bc) return;
    const double t0 = comm_begin(d);
    d->bc(d->user, buf, bytes, root);
    comm_end(d, t0, d->rank == root ? 0.0 : (double)bytes);
}

void sfp_gather_rows(sfp_dev* d, uint64_t* dst, const uint64_t* src, const uint32_t* rows, uint32_t count) {
    for (uint32_t i = 0; i < count; ++i)
        memmove(dst + (size_t)i * d->n, src + (size_t)rows[i] * d->n, (size_t)d->n * 8);
}

void sfp_rescale_rows(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* last,
                      uint32_t drop_prime, sfp_limbs m, const uint64_t* qlinv, uint32_t npoly,
                      size_t in_stride, size_t out_stride, size_t last_stride) {
    const uint32_t n = d->n;
    const u64 ql = d->q[drop_prime];
    for (uint32_t p = 0; p < npoly; ++p) {
        const u64* lp = last + p * last_stride;
        const u64* src = in + p * in_stride;
        u64* dst = out + p * out_stride;
#pragma omp parallel for schedule(static)
        for (uint32_t i = 0; i < m.count; ++i) {
            const uint32_t pi = pidx(m, i);
            const u64 q = d->q[pi];
            u64* row = (u64*)malloc((size_t)n * 8);
            const u64 qlmod = ql % q;
            for (uint32_t x = 0; x < n; ++x) {
                u64 v = lp[x];
                u64 r = v % q;
                if (v > (ql >> 1)) r = sb(r, qlmod, q);
                row[x] = r;
            }
            ntt_fwd(d, row, pi);
            const size_t o = (size_t)i * n;
            for (uint32_t x = 0; x < n; ++x) dst[o + x] = mm(sb(src[o + x], row[x], q), qlinv[i], q);
            free(row);
        }
    }
}

void sfp_ks_inner_map(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                      size_t ext_stride, const uint64_t* key, uint32_t beta, sfp_limbs pm,
                      uint32_t keyQ, uint32_t key_rows, int accum) {
    const uint32_t n = d->n;
#pragma omp parallel for schedule(static)
    for (uint32_t t = 0; t < pm.count; ++t) {
        const uint32_t kr = keyQ == SFP_KEY_ROW_BY_PRIME ? sfp_key_row(&d->kg, pidx(pm, t))
                                                         : (t < pm.split ? t : keyQ + (t - pm.split));
        const u64 q = d->q[pidx(pm, t)];
        for (uint32_t x = 0; x < n; ++x) {
            u128 s0 = 0, s1 = 0;
            for (uint32_t j = 0; j < beta; ++j) {
                u64 e = ext[j * ext_stride + (size_t)t * n + x];
                const u64* kb = key + (size_t)j * 2 * key_rows * n;
                const u64* ka = kb + (size_t)key_rows * n;
                s0 += (u128)e * kb[(size_t)kr * n + x];
                s1 += (u128)e * ka[(size_t)kr * n + x];
            }
            if (accum) {
                s0 += acc0[(size_t)t * n + x];
                s1 += acc1[(size_t)t * n + x];
            }
            acc0[(size_t)t * n + x] = (u64)(s0 % q);
            acc1[(size_t)t * n + x] = (u64)(s1 % q);
        }
    }
}
