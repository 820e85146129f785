// extern "C" boundary (include/sfhe.h) over the lbcrypto-compatible engine.
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <mutex>
#include <sstream>
#include <streambuf>
#include <string>

#include "../../include/sfhe.h"
#include "algo/coefficients.h"
#include "algo/comparison.h"
#include "algo/encryption.h"
#include "algo/rotation.h"
#include "algo/sign.h"
#include "algo/sort_algo.h"
#include "algo/kway_adapter.h"
#include "core/openfhe.h"
#include "core/state.h"

using namespace lbcrypto;
using Ct = Ciphertext<DCRTPoly>;

struct sfhe_ctx {
    CryptoContext<DCRTPoly> cc;
    KeyPair<DCRTPoly> keys;
    bool quiet = false;
};
struct sfhe_ct {
    Ct ct;
};

namespace {

thread_local std::string g_err;

struct NullBuf : std::streambuf {
    int overflow(int c) override { return c; }
};

// silences std::cout while alive (reference prints inside sort()).  Contexts
// may sort concurrently from several threads (one per lane or per shard rank),
// so the swap is reference-counted under a lock with one shared null buffer:
// a per-object buffer restored out of order would leave std::cout pointing at
// a destroyed stack object.
std::mutex g_quietMu;
int g_quietDepth = 0;
std::streambuf* g_quietOld = nullptr;
NullBuf g_nullBuf;

struct Quiet {
    bool on;
    explicit Quiet(bool q) : on(q) {
        if (!on) return;
        std::lock_guard<std::mutex> g(g_quietMu);
        if (g_quietDepth++ == 0) g_quietOld = std::cout.rdbuf(&g_nullBuf);
    }
    ~Quiet() {
        if (!on) return;
        std::lock_guard<std::mutex> g(g_quietMu);
        if (--g_quietDepth == 0) std::cout.rdbuf(g_quietOld);
    }
};

template <class F>
int guard(F&& f) {
    try {
        f();
        return SFHE_OK;
    } catch (const OpenFHEException& e) {
        g_err = e.what();
        return std::string(e.what()).find("device") != std::string::npos ? SFHE_EDEVICE
                                                                          : SFHE_ESCHEME;
    } catch (const std::invalid_argument& e) {
        g_err = e.what();
        return SFHE_EINVAL;
    } catch (const std::exception& e) {
        g_err = e.what();
        return SFHE_ESCHEME;
    }
}

#define REQUIRE(cond, msg)                    \
    do {                                      \
        if (!(cond)) {                        \
            g_err = msg;                      \
            return SFHE_EINVAL;               \
        }                                     \
    } while (0)

sfhe_ct* wrap(Ct c) { return new sfhe_ct{std::move(c)}; }

SignConfig cfgOf(int n, int dg, int df) { return SignConfig(CompositeSignConfig(n, dg, df)); }

struct SorterBase {
    virtual ~SorterBase() = default;
    virtual Ct sort(const Ct& in, SignConfig& cfg) = 0;
    virtual Ct rank(const Ct& in, SignConfig& cfg) = 0;
    virtual Ct place(const Ct& rank, const Ct& in) = 0;
    virtual Ct hybrid1(const Ct& in, SignConfig& cfg, const PrivateKey<DCRTPoly>& sk) = 0;
    virtual Ct hybrid(const Ct& in, SignConfig& cfg, const PrivateKey<DCRTPoly>& sk, int variant) = 0;
    virtual Ct place2N(const Ct& rank, const Ct& in) = 0;
    virtual Ct bitonic(const Ct& in, SignConfig& cfg) = 0;
    virtual size_t graphNodes() const = 0;
    virtual bool graphFamilyTime(uint32_t family, int reps, double* ms, uint64_t* launches, double* bytes) = 0;
};

template <int N>
struct Sorter : SorterBase {
    DirectSort<N> ds;
    std::unique_ptr<BitonicSort<N>> bs;  // built on first use (its mask memo lives across sorts)
    CryptoContext<DCRTPoly> cc_;
    PublicKey<DCRTPoly> pk_;
    std::vector<int> rot_;
    std::shared_ptr<Encryption> enc_;
    Sorter(CryptoContext<DCRTPoly> cc, PublicKey<DCRTPoly> pk, std::vector<int> rot,
           std::shared_ptr<Encryption> enc)
        : ds(cc, pk, rot, enc), cc_(cc), pk_(pk), rot_(rot), enc_(enc) {}
    Ct bitonic(const Ct& in, SignConfig& cfg) override {
        if (!bs) bs = std::make_unique<BitonicSort<N>>(cc_, pk_, rot_, enc_);
        return bs->sort(in, SignFunc::CompositeSign, cfg);
    }
    Ct sort(const Ct& in, SignConfig& cfg) override { return ds.sort(in, SignFunc::CompositeSign, cfg); }
    Ct rank(const Ct& in, SignConfig& cfg) override {
        return ds.constructRank(in, SignFunc::CompositeSign, cfg);
    }
    Ct place(const Ct& r, const Ct& in) override { return ds.rotationIndexCheckN(r, in); }
    Ct hybrid1(const Ct& in, SignConfig& cfg, const PrivateKey<DCRTPoly>& sk) override {
        return ds.sort_hybrid1(in, SignFunc::CompositeSign, cfg, sk);
    }
    Ct hybrid(const Ct& in, SignConfig& cfg, const PrivateKey<DCRTPoly>& sk, int variant) override {
        return variant == 2 ? ds.sort_hybrid2(in, SignFunc::CompositeSign, cfg, sk)
                            : ds.sort_hybrid(in, SignFunc::CompositeSign, cfg, sk);
    }
    Ct place2N(const Ct& r, const Ct& in) override { return ds.rotationIndexCheck2N(r, in); }
    size_t graphNodes() const override { return ds.graphNodes(); }
    bool graphFamilyTime(uint32_t family, int reps, double* ms, uint64_t* launches, double* bytes) override {
        return ds.graphFamilyTime(family, reps, ms, launches, bytes);
    }
};

template <int N>
int decomposeN(const std::vector<int>& keys, int r, int wrap, int algo, int32_t* v, int32_t* s,
               size_t cap, size_t* count) {
    Decomposer<N> d(keys);
    auto steps = d.decompose(r, wrap, algo == 0 ? DecomposeAlgo::NAF
                                      : algo == 1 ? DecomposeAlgo::BNAF
                                                  : DecomposeAlgo::BINARY);
    if (count) *count = steps.size();
    for (size_t i = 0; i < steps.size() && i < cap; ++i) {
        v[i] = steps[i].value;
        s[i] = steps[i].stepSize;
    }
    return SFHE_OK;
}

bool validN(uint32_t N) {
    return N >= 4 && N <= 1024 && (N & (N - 1)) == 0;
}

}  // namespace

struct sfhe_sorter {
    sfhe_ctx* ctx;
    std::unique_ptr<SorterBase> impl;
};

extern "C" {

int sfhe_abi_version(void) { return SFHE_ABI_VERSION; }
const char* sfhe_last_error(void) { return g_err.c_str(); }
const char* sfhe_backend(void) { return sfp_backend_name(); }

void sfhe_params_default(sfhe_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof *p);
    p->mult_depth = 1;
    p->scaling_mod_size = 40;
    p->first_mod_size = 60;
    p->security_level = SFHE_HESTD_128_CLASSIC;
    p->seed = 0x5eed5eed2025ULL;
    p->scaling_technique = SFHE_FLEXIBLEAUTOEXT;
}

int sfhe_context_create(const sfhe_params* p, sfhe_ctx** out) {
    REQUIRE(p && out, "null argument");
    return guard([&] {
        CCParams<CryptoContextCKKSRNS> P;
        P.SetMultiplicativeDepth(p->mult_depth);
        P.SetScalingModSize(p->scaling_mod_size);
        P.SetFirstModSize(p->first_mod_size ? p->first_mod_size : 60);
        P.SetBatchSize(p->batch_size);
        P.SetRingDim(p->ring_dim);
        P.SetSecurityLevel(p->security_level == SFHE_HESTD_NOTSET ? HEStd_NotSet : HEStd_128_classic);
        P.SetNumLargeDigits(p->num_large_digits);
        P.SetDevice(p->device);
        P.SetSeed(p->seed);
        if (p->scaling_technique != 0 && p->scaling_technique != SFHE_FLEXIBLEAUTO &&
            p->scaling_technique != SFHE_FLEXIBLEAUTOEXT)
            throw std::invalid_argument("scaling_technique must be FLEXIBLEAUTO or FLEXIBLEAUTOEXT");
        P.SetScalingTechnique(p->scaling_technique == SFHE_FLEXIBLEAUTO ? FLEXIBLEAUTO
                                                                         : FLEXIBLEAUTOEXT);
        auto c = std::make_unique<sfhe_ctx>();
        c->cc = GenCryptoContext(P);
        c->cc->Enable(PKE);
        c->cc->Enable(KEYSWITCH);
        c->cc->Enable(LEVELEDSHE);
        c->cc->Enable(ADVANCEDSHE);
        *out = c.release();
    });
}

void sfhe_context_destroy(sfhe_ctx* c) { delete c; }

int sfhe_keygen(sfhe_ctx* c) {
    REQUIRE(c, "null context");
    return guard([&] {
        c->keys = c->cc->KeyGen();
        c->cc->EvalMultKeyGen(c->keys.secretKey);
    });
}

int sfhe_rotate_keygen(sfhe_ctx* c, const int32_t* idx, size_t count) {
    REQUIRE(c && (idx || !count), "null argument");
    REQUIRE(c->keys.secretKey, "sfhe_keygen must be called first");
    return guard([&] { c->cc->EvalRotateKeyGen(c->keys.secretKey, std::vector<int32_t>(idx, idx + count)); });
}

int sfhe_context_info(sfhe_ctx* c, uint32_t* n, uint32_t* depth, uint32_t* nq, uint32_t* np,
                      uint32_t* dnum) {
    REQUIRE(c, "null context");
    const SfheContextState* s = c->cc->state();
    if (n) *n = s->n;
    if (depth) *depth = s->L;
    if (nq) *nq = s->Lq;
    if (np) *np = s->K;
    if (dnum) *dnum = s->dnum;
    return SFHE_OK;
}

int sfhe_set_plaintext_cache(sfhe_ctx* c, int on) {
    REQUIRE(c, "null context");
    return guard([&] { c->cc->SetPlaintextCache(on != 0); });
}

int sfhe_set_quiet(sfhe_ctx* c, int q) {
    REQUIRE(c, "null context");
    c->quiet = q != 0;
    return SFHE_OK;
}

int sfhe_sync(sfhe_ctx* c) {
    REQUIRE(c, "null context");
    return guard([&] { c->cc->Synchronize(); });
}

int sfhe_op_stats(sfhe_ctx* c, uint64_t* counts, double* bytes, int reset) {
    REQUIRE(c, "null context");
    auto s = c->cc->GetOpStats();
    if (counts) {
        uint64_t v[9] = {s.keyswitch, s.rescale, s.tensor,  s.ptmult,    s.constmult,
                         s.add,       s.automorph, s.ntt_limbs, s.wsum_terms};
        std::memcpy(counts, v, sizeof v);
    }
    if (bytes) *bytes = s.algo_bytes;
    if (reset) c->cc->ResetOpStats();
    return SFHE_OK;
}

int sfhe_bootstrap_graphs(sfhe_ctx* c, uint64_t* count) {
    REQUIRE(c && count, "null argument");
    *count = c->cc->BootstrapGraphs();
    return SFHE_OK;
}

int sfhe_encode_counts(sfhe_ctx* c, uint64_t* device, uint64_t* host) {
    REQUIRE(c && device && host, "null argument");
    auto s = c->cc->GetOpStats();
    *device = s.dev_encodes;
    *host = s.host_encodes;
    return SFHE_OK;
}

int sfhe_encrypt(sfhe_ctx* c, const double* v, size_t len, uint32_t slots, uint32_t level,
                 sfhe_ct** out) {
    REQUIRE(c && out && (v || !len), "null argument");
    REQUIRE(c->keys.publicKey, "sfhe_keygen must be called first");
    return guard([&] {
        auto pt = c->cc->MakeCKKSPackedPlaintext(std::vector<double>(v, v + len), 1, level, nullptr, slots);
        *out = wrap(c->cc->Encrypt(c->keys.publicKey, pt));
    });
}

int sfhe_decrypt(sfhe_ctx* c, const sfhe_ct* ct, double* out, size_t cap, size_t* len) {
    REQUIRE(c && ct, "null argument");
    REQUIRE(c->keys.secretKey, "no secret key");
    return guard([&] {
        Plaintext pt;
        c->cc->Decrypt(c->keys.secretKey, ct->ct, &pt);
        const auto& v = pt->GetRealPackedValue();
        if (len) *len = v.size();
        for (size_t i = 0; i < v.size() && i < cap; ++i) out[i] = v[i];
    });
}

void sfhe_ct_free(sfhe_ct* ct) { delete ct; }

int sfhe_ct_clone(const sfhe_ct* ct, sfhe_ct** out) {
    REQUIRE(ct && out, "null argument");
    return guard([&] { *out = wrap(ct->ct->Clone()); });
}

int sfhe_ct_info(const sfhe_ct* ct, uint32_t* level, uint32_t* slots, uint32_t* limbs) {
    REQUIRE(ct, "null ciphertext");
    if (level) *level = ct->ct->GetLevel();
    if (slots) *slots = ct->ct->GetSlots();
    if (limbs) *limbs = ct->ct->GetNumLimbs();
    return SFHE_OK;
}

int sfhe_ct_set_slots(sfhe_ct* ct, uint32_t slots) {
    REQUIRE(ct && slots && !(slots & (slots - 1)), "slots must be a power of two");
    ct->ct->SetSlots(slots);
    return SFHE_OK;
}

int sfhe_ct_download(sfhe_ctx* c, const sfhe_ct* ct, uint64_t* out, size_t cap) {
    REQUIRE(c && ct && out, "null argument");
    const size_t n = c->cc->GetRingDimension();
    const size_t L = ct->ct->GetNumLimbs();
    REQUIRE(cap >= 2 * L * n, "output buffer too small");
    return guard([&] { c->cc->DownloadRows(ct->ct, out); });
}

#define BINOP(name, expr)                                                           \
    int name(sfhe_ctx* c, const sfhe_ct* a, const sfhe_ct* b, sfhe_ct** out) {       \
        REQUIRE(c && a && b && out, "null argument");                               \
        return guard([&] { *out = wrap(expr); });                                   \
    }
BINOP(sfhe_eval_add, c->cc->EvalAdd(a->ct, b->ct))
BINOP(sfhe_eval_sub, c->cc->EvalSub(a->ct, b->ct))
BINOP(sfhe_eval_mult, c->cc->EvalMult(a->ct, b->ct))

int sfhe_eval_add_const(sfhe_ctx* c, const sfhe_ct* a, double k, sfhe_ct** out) {
    REQUIRE(c && a && out, "null argument");
    return guard([&] { *out = wrap(c->cc->EvalAdd(a->ct, k)); });
}
int sfhe_eval_mult_const(sfhe_ctx* c, const sfhe_ct* a, double k, sfhe_ct** out) {
    REQUIRE(c && a && out, "null argument");
    return guard([&] { *out = wrap(c->cc->EvalMult(a->ct, k)); });
}
int sfhe_eval_mult_plain(sfhe_ctx* c, const sfhe_ct* a, const double* v, size_t len,
                         uint32_t slots, sfhe_ct** out) {
    REQUIRE(c && a && out && (v || !len), "null argument");
    return guard([&] {
        auto pt = c->cc->MakeCKKSPackedPlaintext(std::vector<double>(v, v + len), 1,
                                                 a->ct->GetLevel(), nullptr, slots);
        *out = wrap(c->cc->EvalMult(a->ct, pt));
    });
}
int sfhe_eval_rotate(sfhe_ctx* c, const sfhe_ct* a, int32_t r, sfhe_ct** out) {
    REQUIRE(c && a && out, "null argument");
    return guard([&] { *out = wrap(c->cc->EvalRotate(a->ct, r)); });
}
int sfhe_eval_rotate_sum(sfhe_ctx* c, const sfhe_ct* const* a, const int32_t* r, size_t count, sfhe_ct** out) {
    REQUIRE(c && a && r && out && count, "null argument");
    for (size_t k = 0; k < count; ++k) REQUIRE(a[k], "null argument");
    return guard([&] {
        std::vector<Ciphertext<DCRTPoly>> v;
        for (size_t k = 0; k < count; ++k) v.push_back(a[k]->ct);
        *out = wrap(c->cc->EvalRotateSum(v, std::vector<int32_t>(r, r + count)));
    });
}
int sfhe_bootstrap_setup(sfhe_ctx* c, uint32_t budget_c2s, uint32_t budget_s2c, uint32_t slots) {
    REQUIRE(c, "null argument");
    REQUIRE(c->keys.secretKey, "sfhe_keygen must be called first");
    return guard([&] {
        c->cc->EvalBootstrapSetup({budget_c2s, budget_s2c}, {0, 0}, slots);
        c->cc->EvalBootstrapKeyGen(c->keys.secretKey, slots);
    });
}
int sfhe_bootstrap_depth(sfhe_ctx* c, uint32_t budget_c2s, uint32_t budget_s2c, uint32_t slots, uint32_t* depth) {
    REQUIRE(c && depth, "null argument");
    return guard([&] { *depth = c->cc->GetBootstrapDepth({budget_c2s, budget_s2c}, slots); });
}
int sfhe_bootstrap(sfhe_ctx* c, const sfhe_ct* a, uint32_t iterations, uint32_t precision, sfhe_ct** out) {
    REQUIRE(c && a && out, "null argument");
    return guard([&] { *out = wrap(c->cc->EvalBootstrap(a->ct, iterations, precision)); });
}
int sfhe_eval_chebyshev(sfhe_ctx* c, const sfhe_ct* x, const double* coeffs, size_t count,
                        double a, double b, sfhe_ct** out) {
    REQUIRE(c && x && coeffs && count && out, "null argument");
    return guard([&] {
        *out = wrap(c->cc->EvalChebyshevSeriesPS(x->ct, std::vector<double>(coeffs, coeffs + count), a, b));
    });
}

int sfhe_sign(sfhe_ctx* c, const sfhe_ct* x, int n, int dg, int df, sfhe_ct** out) {
    REQUIRE(c && x && out, "null argument");
    REQUIRE(n == 3 || n == 4, "composite sign degree n must be 3 or 4");
    return guard([&] { *out = wrap(sign(x->ct, c->cc, SignFunc::CompositeSign, cfgOf(n, dg, df))); });
}

int sfhe_compare(sfhe_ctx* c, const sfhe_ct* a, const sfhe_ct* b, int n, int dg, int df,
                 sfhe_ct** out) {
    REQUIRE(c && a && b && out, "null argument");
    REQUIRE(n == 3 || n == 4, "composite sign degree n must be 3 or 4");
    return guard([&] {
        Comparison cmp;
        auto cfg = cfgOf(n, dg, df);
        *out = wrap(cmp.compare(c->cc, a->ct, b->ct, SignFunc::CompositeSign, cfg));
    });
}

int sfhe_direct_sort_params(uint32_t N, uint32_t* depth, int32_t* rot, size_t cap, size_t* count) {
    const sfhe::SizeParams* p = sfhe::sizeParams((int)N);
    REQUIRE(p, "N has no DirectSort size parameters (reference table: 4 .. 2048)");
    return guard([&] {
        const auto& r = p->rotations;
        if (depth) *depth = (uint32_t)p->multDepth;
        if (count) *count = r.size();
        for (size_t i = 0; i < r.size() && i < cap && rot; ++i) rot[i] = r[i];
    });
}

int sfhe_doubled_sinc_coeffs(uint32_t N, double* out, size_t cap, size_t* count) {
    REQUIRE(validN(N), "N must be a power of two in [4, 1024]");
    return guard([&] {
        const auto& v = sfhe::doubledSincCoefficients((int)N);
        if (count) *count = v.size();
        for (size_t i = 0; i < v.size() && i < cap && out; ++i) out[i] = v[i];
    });
}

int sfhe_sorter_create(sfhe_ctx* c, uint32_t N, int debug, sfhe_sorter** out) {
    return sfhe_sorter_create_rot(c, N, debug, nullptr, 0, out);
}

int sfhe_sorter_create_rot(sfhe_ctx* c, uint32_t N, int debug, const int32_t* rotations, size_t nrot,
                           sfhe_sorter** out) {
    REQUIRE(c && out, "null argument");
    REQUIRE(validN(N), "N must be a power of two in [4, 1024]");
    REQUIRE(c->keys.publicKey, "sfhe_keygen must be called first");
    REQUIRE(!nrot || rotations, "null rotation list");
    return guard([&] {
        std::shared_ptr<Encryption> enc =
            debug ? std::shared_ptr<Encryption>(std::make_shared<DebugEncryption>(c->cc, c->keys))
                  : std::make_shared<Encryption>(c->cc, c->keys.publicKey);
        const auto rot = rotations ? std::vector<int>(rotations, rotations + nrot)
                                   : sfhe::sizeParams((int)N)->rotations;
        auto s = std::make_unique<sfhe_sorter>();
        s->ctx = c;
        switch (N) {
#define CASE(K) \
    case K: s->impl.reset(new Sorter<K>(c->cc, c->keys.publicKey, rot, enc)); break;
            CASE(4) CASE(8) CASE(16) CASE(32) CASE(64) CASE(128) CASE(256) CASE(512) CASE(1024)
#undef CASE
        }
        *out = s.release();
    });
}

void sfhe_sorter_destroy(sfhe_sorter* s) { delete s; }

int sfhe_sorter_sort(sfhe_sorter* s, sfhe_ct* in, int n, int dg, int df, sfhe_ct** out) {
    REQUIRE(s && in && out, "null argument");
    return guard([&] {
        Quiet q(s->ctx->quiet);
        auto cfg = cfgOf(n, dg, df);
        *out = wrap(s->impl->sort(in->ct, cfg));
    });
}

int sfhe_sorter_rank(sfhe_sorter* s, const sfhe_ct* in, int n, int dg, int df, sfhe_ct** out) {
    REQUIRE(s && in && out, "null argument");
    return guard([&] {
        auto cfg = cfgOf(n, dg, df);
        *out = wrap(s->impl->rank(in->ct, cfg));
    });
}

int sfhe_sorter_place(sfhe_sorter* s, const sfhe_ct* rank, sfhe_ct* in, sfhe_ct** out) {
    REQUIRE(s && rank && in && out, "null argument");
    return guard([&] { *out = wrap(s->impl->place(rank->ct, in->ct)); });
}

int sfhe_sorter_sort_hybrid1(sfhe_sorter* s, sfhe_ct* in, int n, int dg, int df, sfhe_ct** out) {
    REQUIRE(s && in && out, "null argument");
    REQUIRE(s->ctx->keys.secretKey, "sfhe_keygen must be called first");
    return guard([&] {
        Quiet q(s->ctx->quiet);
        auto cfg = cfgOf(n, dg, df);
        *out = wrap(s->impl->hybrid1(in->ct, cfg, s->ctx->keys.secretKey));
    });
}

int sfhe_sorter_sort_hybrid(sfhe_sorter* s, sfhe_ct* in, int variant, int n, int dg, int df, sfhe_ct** out) {
    REQUIRE(s && in && out, "null argument");
    REQUIRE(variant == 0 || variant == 2, "variant must be 0 (sort_hybrid) or 2 (sort_hybrid2)");
    REQUIRE(s->ctx->keys.secretKey, "sfhe_keygen must be called first");
    return guard([&] {
        Quiet q(s->ctx->quiet);
        auto cfg = cfgOf(n, dg, df);
        *out = wrap(s->impl->hybrid(in->ct, cfg, s->ctx->keys.secretKey, variant));
    });
}

int sfhe_sorter_place_2n(sfhe_sorter* s, const sfhe_ct* rank, sfhe_ct* in, sfhe_ct** out) {
    REQUIRE(s && rank && in && out, "null argument");
    return guard([&] { *out = wrap(s->impl->place2N(rank->ct, in->ct)); });
}

int sfhe_sorter_sort_bitonic(sfhe_sorter* s, sfhe_ct* in, int n, int dg, int df, sfhe_ct** out) {
    REQUIRE(s && in && out, "null argument");
    REQUIRE(n == 3 || n == 4, "composite sign degree n must be 3 or 4");
    return guard([&] {
        Quiet q(s->ctx->quiet);
        auto cfg = cfgOf(n, dg, df);
        *out = wrap(s->impl->bitonic(in->ct, cfg));
    });
}

int sfhe_save(sfhe_ctx* c, const char* dir) {
    REQUIRE(c && dir, "null argument");
    return guard([&] {
        const std::string d(dir);
        auto put = [&](const std::string& name, auto&& write) {
            std::ofstream f(d + "/" + name, std::ios::binary | std::ios::trunc);
            if (!f.is_open() || !write(f) || !f.good()) throw std::invalid_argument("cannot write " + d + "/" + name);
        };
        put("cc.bin", [&](std::ostream& f) { return Serial::Serialize(c->cc, f, SerType::BINARY); });
        put("pub.bin", [&](std::ostream& f) { return Serial::Serialize(c->keys.publicKey, f, SerType::BINARY); });
        if (c->keys.secretKey)
            put("sk.bin", [&](std::ostream& f) { return Serial::Serialize(c->keys.secretKey, f, SerType::BINARY); });
        // this context's key pair only (other engines in the process keep theirs)
        const std::string tag = KeyTagString(c->cc->KeyTag());
        put("mult.bin", [&](std::ostream& f) {
            return CryptoContextImpl<DCRTPoly>::SerializeEvalMultKey(f, SerType::BINARY, tag);
        });
        put("rot.bin", [&](std::ostream& f) {
            return CryptoContextImpl<DCRTPoly>::SerializeEvalAutomorphismKey(f, SerType::BINARY, tag);
        });
    });
}

int sfhe_load(const char* dir, sfhe_ctx** out) {
    REQUIRE(dir && out, "null argument");
    return guard([&] {
        const std::string d(dir);
        auto get = [&](const std::string& name, bool required, auto&& read) {
            std::ifstream f(d + "/" + name, std::ios::binary);
            if (!f.is_open()) {
                if (required) throw std::invalid_argument("cannot open " + d + "/" + name);
                return;
            }
            if (!read(f)) throw std::invalid_argument("cannot deserialize " + d + "/" + name);
        };
        auto ctx = std::make_unique<sfhe_ctx>();
        get("cc.bin", true, [&](std::istream& f) { return Serial::Deserialize(ctx->cc, f, SerType::BINARY); });
        get("pub.bin", true, [&](std::istream& f) { return Serial::Deserialize(ctx->keys.publicKey, f, SerType::BINARY); });
        get("sk.bin", false, [&](std::istream& f) { return Serial::Deserialize(ctx->keys.secretKey, f, SerType::BINARY); });
        get("mult.bin", true, [&](std::istream& f) { return CryptoContextImpl<DCRTPoly>::DeserializeEvalMultKey(f, SerType::BINARY); });
        get("rot.bin", true, [&](std::istream& f) {
            return CryptoContextImpl<DCRTPoly>::DeserializeEvalAutomorphismKey(f, SerType::BINARY);
        });
        *out = ctx.release();
    });
}

int sfhe_ct_save(sfhe_ctx* c, const sfhe_ct* ct, const char* path) {
    REQUIRE(c && ct && path, "null argument");
    return guard([&] {
        if (!Serial::SerializeToFile(std::string(path), ct->ct, SerType::BINARY))
            throw std::invalid_argument(std::string("cannot write ") + path);
    });
}

int sfhe_ct_load(sfhe_ctx* c, const char* path, sfhe_ct** out) {
    REQUIRE(c && path && out, "null argument");
    return guard([&] {
        Ct ct;
        if (!Serial::DeserializeFromFile(std::string(path), ct, SerType::BINARY))
            throw std::invalid_argument(std::string("cannot read ") + path);
        *out = wrap(ct);
    });
}

int sfhe_kway_sort(sfhe_ctx* c, const sfhe_ct* in, int k, int M, int n, int dg, int df, uint32_t mult_depth,
                   sfhe_ct** out) {
    REQUIRE(c && in && out, "null argument");
    REQUIRE(k == 2 || k == 3 || k == 5, "k must be 2, 3 or 5");
    REQUIRE(M >= 1 && M <= 16, "M out of range");
    REQUIRE(n == 3 || n == 4, "composite sign degree n must be 3 or 4");
    long len = 1;
    for (int i = 0; i < M; ++i) len *= k;
    REQUIRE(len <= (long)in->ct->GetSlots(), "k^M exceeds the ciphertext's slots");
    return guard([&] {
        Quiet q(c->quiet);
        // (the sorter keeps the keys only for its debug decryptions)
        kwaySort::Sorter sorter(c->cc, nullptr, (long)in->ct->GetSlots(), k, M, c->keys.secretKey,
                                c->keys.publicKey);
        SignConfig cfg(CompositeSignConfig(n, dg, df), (int)mult_depth);
        Ct x = in->ct->Clone(), y;
        sorter.sorter(x, y, cfg);
        if (!y) throw OpenFHEException("k-way sorter: no stage schedule for this k");
        *out = wrap(y);
    });
}

}  // extern "C"

namespace {
struct KWayBase {
    virtual ~KWayBase() = default;
    virtual Ct run(const Ct& in, SignConfig& cfg) = 0;
    virtual size_t graphNodes() const = 0;
    virtual bool graphFamilyTime(uint32_t family, int reps, double* ms, uint64_t* launches, double* bytes) = 0;
};
template <int N>
struct KWayImpl : KWayBase {
    KWayAdapter<N> a;
    KWayImpl(sfhe_ctx* c, int k, int M)
        : a(c->cc, c->keys.publicKey, c->keys.secretKey,
            std::make_shared<Encryption>(c->cc, c->keys.publicKey), k, M) {}
    Ct run(const Ct& in, SignConfig& cfg) override { return a.sort(in, SignFunc::CompositeSign, cfg); }
    size_t graphNodes() const override { return a.graphNodes(); }
    bool graphFamilyTime(uint32_t family, int reps, double* ms, uint64_t* launches, double* bytes) override {
        return a.graphFamilyTime(family, reps, ms, launches, bytes);
    }
};
std::unique_ptr<KWayBase> makeKWay(sfhe_ctx* c, uint32_t N, int k, int M) {
    switch (N) {
#define SFHE_KWAY_N(v) \
    case v: return std::make_unique<KWayImpl<v>>(c, k, M);
        SFHE_KWAY_N(4) SFHE_KWAY_N(8) SFHE_KWAY_N(16) SFHE_KWAY_N(32) SFHE_KWAY_N(64) SFHE_KWAY_N(128)
        SFHE_KWAY_N(256) SFHE_KWAY_N(512) SFHE_KWAY_N(1024) SFHE_KWAY_N(9) SFHE_KWAY_N(27) SFHE_KWAY_N(81)
        SFHE_KWAY_N(243) SFHE_KWAY_N(729) SFHE_KWAY_N(25) SFHE_KWAY_N(125) SFHE_KWAY_N(625)
#undef SFHE_KWAY_N
    }
    return nullptr;
}
}  // namespace

struct sfhe_kway {
    sfhe_ctx* ctx;
    std::unique_ptr<KWayBase> impl;
};

extern "C" {

int sfhe_kway_create(sfhe_ctx* c, uint32_t N, int k, int M, sfhe_kway** out) {
    REQUIRE(c && out, "null argument");
    REQUIRE(k == 2 || k == 3 || k == 5, "k must be 2, 3 or 5");
    long len = 1;
    for (int i = 0; i < M && len <= (1 << 20); ++i) len *= k;
    REQUIRE(M >= 1 && len == (long)N, "N must equal k^M");
    return guard([&] {
        auto impl = makeKWay(c, N, k, M);
        if (!impl) throw std::invalid_argument("unsupported N for the k-way network");
        *out = new sfhe_kway{c, std::move(impl)};
    });
}

int sfhe_kway_run(sfhe_kway* s, const sfhe_ct* in, int n, int dg, int df, uint32_t mult_depth, sfhe_ct** out) {
    REQUIRE(s && in && out, "null argument");
    REQUIRE(n == 3 || n == 4, "composite sign degree n must be 3 or 4");
    return guard([&] {
        Quiet q(s->ctx->quiet);
        SignConfig cfg(CompositeSignConfig(n, dg, df), (int)mult_depth);
        *out = wrap(s->impl->run(in->ct, cfg));
    });
}

void sfhe_kway_destroy(sfhe_kway* s) { delete s; }

int sfhe_kway_graph_family_time(sfhe_kway* s, uint32_t family, int reps, double* ms, uint64_t* launches,
                                double* bytes) {
    REQUIRE(s && ms && reps > 0, "null argument");
    REQUIRE(family <= SFHE_KFAM_ALL, "unknown kernel family");
    return guard([&] {
        if (!s->impl->graphFamilyTime(family, reps, ms, launches, bytes))
            throw std::runtime_error("no captured k-way graph with kernels of that family");
    });
}

int sfhe_kway_graph_nodes(const sfhe_kway* s, uint64_t* nodes) {
    REQUIRE(s && nodes, "null argument");
    *nodes = s->impl->graphNodes();
    return SFHE_OK;
}

int sfhe_kway_params(uint32_t N, uint32_t* batch, uint32_t* mult_depth, uint32_t* budget_c2s, uint32_t* budget_s2c,
                     int32_t* rotations, size_t cap, size_t* count) {
    REQUIRE(N >= 2 && N <= (1u << 16), "N out of range");
    uint32_t b = 1;
    while (b < N) b <<= 1;
    if (batch) *batch = b;
    if (mult_depth) *mult_depth = 40;
    if (budget_c2s) *budget_c2s = N <= 128 ? 4 : 5;
    if (budget_s2c) *budget_s2c = N <= 128 ? 4 : 5;
    std::vector<int32_t> r;
    for (uint32_t i = 1; i < N; i *= 2) {
        r.push_back((int32_t)i);
        r.push_back(-(int32_t)i);
    }
    if (count) *count = r.size();
    for (size_t i = 0; i < r.size() && i < cap && rotations; ++i) rotations[i] = r[i];
    return SFHE_OK;
}

int sfhe_hybrid1_params(uint32_t N, uint32_t* mult_depth, int32_t* rotations, size_t cap, size_t* count) {
    REQUIRE(validN(N), "N must be a power of two in [4, 1024]");
    const sfhe::SizeParams* p = sfhe::hybrid1Params((int)N);
    if (mult_depth) *mult_depth = (uint32_t)p->multDepth;
    if (count) *count = p->rotations.size();
    for (size_t i = 0; i < p->rotations.size() && i < cap && rotations; ++i) rotations[i] = p->rotations[i];
    return SFHE_OK;
}

int sfhe_hybrid_params(uint32_t N, int variant, uint32_t* mult_depth, int32_t* rotations, size_t cap,
                       size_t* count) {
    REQUIRE(validN(N), "N must be a power of two in [4, 1024]");
    REQUIRE(variant == 0 || variant == 2, "variant must be 0 (sort_hybrid) or 2 (sort_hybrid2)");
    const sfhe::SizeParams* p = sfhe::hybridParams((int)N, variant);
    if (mult_depth) *mult_depth = (uint32_t)p->multDepth;
    if (count) *count = p->rotations.size();
    for (size_t i = 0; i < p->rotations.size() && i < cap && rotations; ++i) rotations[i] = p->rotations[i];
    return SFHE_OK;
}

int sfhe_sorter_graph_family_time(sfhe_sorter* s, uint32_t family, int reps, double* ms, uint64_t* launches,
                                  double* bytes) {
    REQUIRE(s && ms && reps > 0, "null argument");
    static_assert(SFHE_KFAM_OTHER == SFP_FAM_COUNT && SFHE_KFAM_ALL == SFP_FAM_ALL, "family numbering");
    REQUIRE(family <= SFHE_KFAM_ALL, "unknown kernel family");
    return guard([&] {
        if (!s->impl->graphFamilyTime(family, reps, ms, launches, bytes))
            throw std::runtime_error("no captured sort graph (or no graphs on this backend)");
    });
}

int sfhe_sorter_graph_ntt_time(sfhe_sorter* s, int reps, double* ms, uint64_t* launches, double* bytes) {
    return sfhe_sorter_graph_family_time(s, SFHE_KFAM_NTT, reps, ms, launches, bytes);
}

int sfhe_sorter_graph_nodes(const sfhe_sorter* s, uint64_t* nodes) {
    REQUIRE(s && nodes, "null argument");
    *nodes = s->impl->graphNodes();
    return SFHE_OK;
}

int sfhe_decompose(uint32_t N, const int32_t* keys, size_t nkeys, int32_t rotation, int32_t wrapN,
                   int algo, int32_t* values, int32_t* steps, size_t cap, size_t* count) {
    REQUIRE(validN(N) && keys && nkeys && wrapN > 0, "bad argument");
    std::vector<int> k(keys, keys + nkeys);
    return guard([&] {
        switch (N) {
#define CASE(K) \
    case K: decomposeN<K>(k, rotation, wrapN, algo, values, steps, cap, count); break;
            CASE(4) CASE(8) CASE(16) CASE(32) CASE(64) CASE(128) CASE(256) CASE(512) CASE(1024)
#undef CASE
        }
    });
}

int sfhe_debug_decrypt_coeffs(sfhe_ctx* c, const sfhe_ct* ct, double* out, size_t cap) {
    REQUIRE(c && ct && out, "null argument");
    REQUIRE(c->keys.secretKey, "no secret key");
    REQUIRE(!c->cc->IsSharded(), "debug decrypt needs an unsharded context");
    const size_t n = c->cc->GetRingDimension();
    REQUIRE(cap >= n, "output buffer too small");
    return guard([&] {
        auto* s = c->cc->state();
        c->cc->Settle(ct->ct);
        auto t = s->alloc(n);
        const sfp_limbs q{1, 1, 0, 0};
        sfp_mul_add(s->dev, t->ptr, ct->ct->c1, c->keys.secretKey->s->ptr, ct->ct->c0, q);
        sfp_ntt(s->dev, t->ptr, q, 1);
        std::vector<uint64_t> h(n);
        sfp_d2h(s->dev, h.data(), t->ptr, n * 8);
        const uint64_t q0 = s->primes[0];
        for (size_t i = 0; i < n; ++i) out[i] = h[i] > q0 / 2 ? -(double)(q0 - h[i]) : (double)h[i];
    });
}

int sfhe_kernel_timing(sfhe_ctx* c, uint32_t family, uint32_t period) {
    REQUIRE(c, "null context");
    REQUIRE(family < SFP_FAM_COUNT, "unknown kernel family");
    return guard([&] {
        OpLock g(c->cc->state());
        sfp_prof_set(c->cc->state()->dev, family, period);
    });
}

int sfhe_serialize_lanes(sfhe_ctx* c, int on) {
    REQUIRE(c, "null context");
    return guard([&] {
        OpLock g(c->cc->state());
        sfp_serialize(c->cc->state()->dev, on);
    });
}

int sfhe_stack_stats(sfhe_ctx* c, uint64_t* merged, uint64_t* single) {
    REQUIRE(c, "null context");
    return guard([&] {
        OpLock g(c->cc->state());
        sfp_stack_stats(c->cc->state()->dev, merged, single);
    });
}

int sfhe_comm_stats_reset(sfhe_ctx* c, int timed) {
    REQUIRE(c, "null context");
    return guard([&] {
        OpLock g(c->cc->state());
        sfp_comm_stats_reset(c->cc->state()->dev, timed);
    });
}

int sfhe_comm_stats(sfhe_ctx* c, uint64_t* calls, double* bytes, double* ms) {
    REQUIRE(c, "null context");
    return guard([&] {
        OpLock g(c->cc->state());
        sfp_comm_stats(c->cc->state()->dev, calls, bytes, ms);
    });
}

int sfhe_kernel_timing_read(sfhe_ctx* c, uint32_t family, uint64_t* launches, uint64_t* timed,
                            double* ms, double* bytes) {
    REQUIRE(c, "null context");
    REQUIRE(family < SFP_FAM_COUNT, "unknown kernel family");
    return guard([&] {
        OpLock g(c->cc->state());
        sfp_prof_read(c->cc->state()->dev, family, launches, timed, ms, bytes);
    });
}

int sfhe_context_primes(sfhe_ctx* c, uint64_t* out, size_t cap, size_t* count) {
    REQUIRE(c, "null context");
    const auto& p = c->cc->state()->primes;
    if (count) *count = p.size();
    for (size_t i = 0; i < p.size() && i < cap && out; ++i) out[i] = p[i];
    return SFHE_OK;
}

int sfhe_live_contexts(void) { return CryptoContextImpl<DCRTPoly>::LiveContexts(); }

int sfhe_pool_bytes(sfhe_ctx* c, uint64_t* bytes) {
    REQUIRE(c && bytes, "null argument");
    *bytes = c->cc->GetOpStats().pool_bytes;
    return SFHE_OK;
}

// ---- limb sharding ----
int sfhe_comm_uid(uint8_t uid[128]) {
    REQUIRE(uid, "null argument");
    if (sfp_comm_uid(uid) != 0) {
        g_err = std::string("no RCCL communicator in the ") + sfp_backend_name() + " backend";
        return SFHE_ENOTIMPL;
    }
    return SFHE_OK;
}

int sfhe_shard_rccl(sfhe_ctx* c, int rank, int world, const uint8_t uid[128]) {
    REQUIRE(c && uid, "null argument");
    REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank / world");
    REQUIRE(!c->keys.secretKey, "shard the context before sfhe_keygen");
    REQUIRE(!c->cc->IsSharded(), "context already sharded");
    return guard([&] {
        auto* s = c->cc->state();
        if (sfp_comm_init_rccl(s->dev, rank, world, uid) != 0) {
            const char* e = sfp_last_error(s->dev);
            throw OpenFHEException(std::string("device error: RCCL communicator: ") + (e ? e : "init failed"));
        }
        // a one-rank communicator runs the sharded path too: its all-gathers
        // and broadcasts go through RCCL (single-GPU validation)
        c->cc->EnableSharding(rank, world, true);
    });
}

int sfhe_shard_host(sfhe_ctx* c, int rank, int world, sfhe_allgather_fn ag, sfhe_bcast_fn bc, void* user) {
    REQUIRE(c && ag && bc, "null argument");
    REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank / world");
    REQUIRE(!c->keys.secretKey, "shard the context before sfhe_keygen");
    REQUIRE(!c->cc->IsSharded(), "context already sharded");
    return guard([&] {
        c->cc->EnableSharding(rank, world);
        sfp_comm_set_host(c->cc->state()->dev, rank, world, ag, bc, user);
    });
}

int sfhe_shard_tail(const sfhe_ctx* c, uint32_t* limbs) {
    REQUIRE(c && limbs, "null argument");
    *limbs = c->cc->ShardTailLimbs();
    return SFHE_OK;
}

int sfhe_key_rows(const sfhe_ctx* c, uint32_t* rows) {
    REQUIRE(c && rows, "null argument");
    *rows = c->cc->SwitchKeyRows();
    return SFHE_OK;
}

// ---- batch groups ----
int sfhe_groups_rccl(sfhe_ctx* c, int group, int groups, const uint8_t uid[128]) {
    REQUIRE(c && uid, "null argument");
    REQUIRE(groups >= 1 && group >= 0 && group < groups, "bad group / groups");
    REQUIRE(!c->keys.secretKey, "set the batch groups before sfhe_keygen");
    REQUIRE(c->cc->BatchGroups() == 1, "batch groups already set");
    return guard([&] {
        auto* s = c->cc->state();
        if (sfp_group_init_rccl(s->dev, group, groups, uid) != 0) {
            const char* e = sfp_last_error(s->dev);
            throw OpenFHEException(std::string("device error: RCCL group communicator: ") +
                                   (e ? e : "init failed"));
        }
        // a one-group communicator still gathers every part (through RCCL)
        c->cc->EnableBatchGroups(group, groups, true);
    });
}

int sfhe_groups_host(sfhe_ctx* c, int group, int groups, sfhe_allgather_fn ag, void* user) {
    REQUIRE(c && ag, "null argument");
    REQUIRE(groups >= 1 && group >= 0 && group < groups, "bad group / groups");
    REQUIRE(!c->keys.secretKey, "set the batch groups before sfhe_keygen");
    REQUIRE(c->cc->BatchGroups() == 1, "batch groups already set");
    return guard([&] {
        c->cc->EnableBatchGroups(group, groups, true);
        sfp_group_set_host(c->cc->state()->dev, group, groups, ag, user);
    });
}

int sfhe_groups(const sfhe_ctx* c, int* group, int* groups) {
    REQUIRE(c && group && groups, "null argument");
    *group = c->cc->BatchGroup();
    *groups = c->cc->BatchGroups();
    return SFHE_OK;
}

}  // extern "C"
