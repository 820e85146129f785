// Serialization of contexts, keys and ciphertexts (the OpenFHE surface the
// reference's src/sort.h:31-102 and src/main.cpp:9-44 use: Serial::
// {Serialize,Deserialize}{,To,From}File, CryptoContextImpl::{Serialize,
// Deserialize}Eval{Mult,Automorphism}Key).
//
// Record layout (little-endian):  "SFHE" | u32 version | u32 kind | u64
// fingerprint | body.  A context record carries the parameters and the prime
// chain (the chain is re-derived on load and must match); key and
// ciphertext records carry their key pair's tag, then their device words,
// whose counts are checked against the context's sizes before anything is
// allocated.  A key record binds to the context this thread deserialized
// last when its fingerprint matches, else to a context of its fingerprint
// holding no key pair yet (newest first), else to the one holding its own key
// pair; a ciphertext record the other way round (openfhe.h, Serialize*Key).
#include <algorithm>
#include <cstring>
#include <mutex>

#include "openfhe.h"
#include "state.h"

namespace lbcrypto {
namespace {

constexpr uint32_t kVersion = 2;  // 2: key-pair tags in key / ciphertext records
enum RecKind : uint32_t { R_CC = 1, R_PK = 2, R_SK = 3, R_CT = 4, R_MULT = 5, R_ROT = 6 };

std::mutex g_regMu;
std::vector<std::weak_ptr<CryptoContextImpl<DCRTPoly>>> g_registry;

// The live context a record of fingerprint fp and key-pair tag `tag` binds
// to: a context holding that key pair, or one holding none yet (which the
// record then claims), in the order `keysFirst` gives; newest first within
// each.  Never a context of another key pair.
// The context the calling thread deserialized last: the key records of one
// load (src/sort.h:31-74 reads the context, then its keys) bind to it first,
// so another live context with the same parameters -- keyless, or holding the
// same key pair -- never receives part of that load.
thread_local std::weak_ptr<CryptoContextImpl<DCRTPoly>> t_loaded;

CryptoContext<DCRTPoly> findContext(uint64_t fp, uint64_t tag, bool freshFirst) {
    std::lock_guard<std::mutex> g(g_regMu);
    if (auto cc = t_loaded.lock()) {
        if (cc->Fingerprint() == fp) {
            SfheContextState* s = cc->state();
            if (freshFirst && s->keyTag == 0) {
                s->keyTag = tag;
                return cc;
            }
            if (tag && s->keyTag == tag) return cc;
        }
    }
    for (int pass = 0; pass < 2; ++pass) {
        const bool wantFresh = (pass == 0) == freshFirst;
        for (auto it = g_registry.rbegin(); it != g_registry.rend(); ++it)
            if (auto cc = it->lock()) {
                if (cc->Fingerprint() != fp) continue;
                SfheContextState* s = cc->state();
                if (wantFresh && s->keyTag == 0) {
                    s->keyTag = tag;
                    return cc;
                }
                if (!wantFresh && tag && s->keyTag == tag) return cc;
            }
    }
    return nullptr;
}


template <class T>
void put(std::ostream& os, const T& v) {
    os.write(reinterpret_cast<const char*>(&v), sizeof v);
}
template <class T>
bool get(std::istream& is, T& v) {
    return (bool)is.read(reinterpret_cast<char*>(&v), sizeof v);
}

void header(std::ostream& os, uint32_t kind, uint64_t fp) {
    os.write("SFHE", 4);
    put(os, kVersion);
    put(os, kind);
    put(os, fp);
}
bool readHeader(std::istream& is, uint32_t want, uint64_t& fp) {
    char m[4];
    uint32_t ver = 0, kind = 0;
    if (!is.read(m, 4) || std::memcmp(m, "SFHE", 4) != 0) return false;
    if (!get(is, ver) || ver != kVersion || !get(is, kind) || kind != want) return false;
    return get(is, fp);
}

bool binaryOnly(SerType::Kind k) {
    if (k != SerType::BINARY) {
        std::cerr << "sfhe: only SerType::BINARY serialization is supported" << std::endl;
        return false;
    }
    return true;
}

SfheContextState* unsharded(const CryptoContext<DCRTPoly>& cc) {
    SfheContextState* s = cc->state();
    if (s->sharded) SFHE_THROW("serialization of a limb-sharded context is not supported");
    return s;
}

// device words of a buffer -> stream (u64 count, then the words)
void putWords(std::ostream& os, SfheContextState* s, const uint64_t* p, size_t words) {
    std::vector<uint64_t> h(words);
    if (words) sfp_d2h(s->dev, h.data(), p, words * 8);
    put(os, (uint64_t)words);
    os.write(reinterpret_cast<const char*>(h.data()), (std::streamsize)(words * 8));
}
// stream -> a new pooled device buffer of exactly `expect` words (the size
// the context implies: a record of another size is rejected before anything
// is allocated); null on a short record or a failed allocation
DeviceBufferPtr getWords(std::istream& is, SfheContextState* s, size_t expect) {
    uint64_t words = 0;
    if (!get(is, words) || words != expect || !words) return nullptr;
    try {
        std::vector<uint64_t> h(words);
        if (!is.read(reinterpret_cast<char*>(h.data()), (std::streamsize)(words * 8))) return nullptr;
        auto b = s->alloc(words);
        sfp_h2d(s->dev, b->ptr, h.data(), words * 8);
        return b;
    } catch (const std::exception&) {
        return nullptr;
    }
}
// word counts of the key kinds
size_t pkWords(const SfheContextState* s) { return (size_t)(s->Lq + (s->ext ? 1 : 0)) * s->n; }
size_t skWords(const SfheContextState* s) { return (size_t)s->tablePrimes() * s->n; }
size_t switchKeyWords(const SfheContextState* s) { return (size_t)s->dnum * 2 * (s->Lq + s->K) * s->n; }

}  // namespace

void RegisterCryptoContext(const CryptoContext<DCRTPoly>& cc) {
    std::lock_guard<std::mutex> g(g_regMu);
    g_registry.erase(std::remove_if(g_registry.begin(), g_registry.end(), [](auto& w) { return w.expired(); }),
                     g_registry.end());
    g_registry.push_back(cc);
}

const CCParams<CryptoContextCKKSRNS>& CryptoContextImpl<DCRTPoly>::GetParams() const { return st->params; }

uint64_t CryptoContextImpl<DCRTPoly>::Fingerprint() const {
    const SfheContextState* s = st.get();
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
    mix(s->n);
    mix(s->L);
    mix(s->K);
    mix(s->dnum);
    mix(s->ext);
    for (uint64_t p : s->primes) mix(p);
    for (double d : s->scale) {
        uint64_t b;
        std::memcpy(&b, &d, 8);
        mix(b);
    }
    return h;
}

// ---- context ----
bool Serial::Serialize(const CryptoContext<DCRTPoly>& cc, std::ostream& os, SerType::Kind k) {
    if (!binaryOnly(k) || !cc) return false;
    SfheContextState* s = unsharded(cc);
    const auto& p = s->params;
    header(os, R_CC, cc->Fingerprint());
    put(os, p.GetMultiplicativeDepth());
    put(os, p.GetScalingModSize());
    put(os, p.GetFirstModSize());
    put(os, p.GetBatchSize());
    put(os, p.GetRingDim());
    put(os, (int32_t)p.GetSecurityLevel());
    put(os, p.GetNumLargeDigits());
    put(os, (int32_t)p.GetScalingTechnique());
    put(os, (int32_t)p.GetKeySwitchTechnique());
    put(os, p.GetSeed());
    put(os, cc->GetEnabledMask());
    put(os, (uint32_t)s->primes.size());
    for (uint64_t q : s->primes) put(os, q);
    return os.good();
}

bool Serial::Deserialize(CryptoContext<DCRTPoly>& cc, std::istream& is, SerType::Kind k) {
    if (!binaryOnly(k)) return false;
    uint64_t fp = 0;
    if (!readHeader(is, R_CC, fp)) return false;
    uint32_t depth, sms, fms, batch, ring, nld, mask, np;
    int32_t sec, tech, ks;
    uint64_t seed;
    if (!(get(is, depth) && get(is, sms) && get(is, fms) && get(is, batch) && get(is, ring) && get(is, sec) &&
          get(is, nld) && get(is, tech) && get(is, ks) && get(is, seed) && get(is, mask) && get(is, np)))
        return false;
    std::vector<uint64_t> primes(np);
    for (auto& q : primes)
        if (!get(is, q)) return false;
    CCParams<CryptoContextCKKSRNS> p;
    p.SetMultiplicativeDepth(depth);
    p.SetScalingModSize(sms);
    p.SetFirstModSize(fms);
    p.SetBatchSize(batch);
    p.SetRingDim(ring);
    p.SetSecurityLevel((SecurityLevel)sec);
    p.SetNumLargeDigits(nld);
    p.SetScalingTechnique((ScalingTechnique)tech);
    p.SetKeySwitchTechnique((KeySwitchTechnique)ks);
    p.SetSeed(seed);
    // always a context of its own: the key records that follow bind to it
    // (a live context with the same parameters keeps its own key pair)
    auto c = GenCryptoContext(p);
    c->Enable(mask);
    if (c->state()->primes != primes || c->Fingerprint() != fp) {
        std::cerr << "sfhe: deserialized context does not reproduce the serialized prime chain" << std::endl;
        return false;
    }
    cc = c;
    t_loaded = c;
    return true;
}

// ---- keys ----
bool Serial::Serialize(const PublicKey<DCRTPoly>& pk, std::ostream& os, SerType::Kind k) {
    if (!binaryOnly(k) || !pk) return false;
    SfheContextState* s = unsharded(pk->cc);
    OpLock g(s);
    header(os, R_PK, pk->cc->Fingerprint());
    put(os, pk->tag);
    putWords(os, s, pk->b->ptr, pk->b->words);
    putWords(os, s, pk->a->ptr, pk->a->words);
    return os.good();
}

bool Serial::Deserialize(PublicKey<DCRTPoly>& pk, std::istream& is, SerType::Kind k) {
    if (!binaryOnly(k)) return false;
    uint64_t fp = 0;
    uint64_t tag = 0;
    if (!readHeader(is, R_PK, fp) || !get(is, tag) || !tag) return false;
    auto cc = findContext(fp, tag, true);
    if (!cc) {
        std::cerr << "sfhe: no live crypto context matches the public key (deserialize the context first)"
                  << std::endl;
        return false;
    }
    SfheContextState* s = unsharded(cc);
    OpLock g(s);
    auto out = std::make_shared<PublicKeyImpl<DCRTPoly>>();
    out->cc = cc;
    out->tag = tag;
    out->b = getWords(is, s, pkWords(s));
    out->a = out->b ? getWords(is, s, pkWords(s)) : nullptr;
    if (!out->a) return false;
    pk = out;
    return true;
}

bool Serial::Serialize(const PrivateKey<DCRTPoly>& sk, std::ostream& os, SerType::Kind k) {
    if (!binaryOnly(k) || !sk) return false;
    SfheContextState* s = unsharded(sk->cc);
    OpLock g(s);
    header(os, R_SK, sk->cc->Fingerprint());
    put(os, sk->tag);
    putWords(os, s, sk->s->ptr, sk->s->words);
    put(os, (uint64_t)sk->ternary.size());
    os.write(reinterpret_cast<const char*>(sk->ternary.data()), (std::streamsize)sk->ternary.size());
    return os.good();
}

bool Serial::Deserialize(PrivateKey<DCRTPoly>& sk, std::istream& is, SerType::Kind k) {
    if (!binaryOnly(k)) return false;
    uint64_t fp = 0;
    uint64_t tag = 0;
    if (!readHeader(is, R_SK, fp) || !get(is, tag) || !tag) return false;
    auto cc = findContext(fp, tag, true);
    if (!cc) return false;
    SfheContextState* s = unsharded(cc);
    OpLock g(s);
    auto out = std::make_shared<PrivateKeyImpl<DCRTPoly>>();
    out->cc = cc;
    out->tag = tag;
    out->s = getWords(is, s, skWords(s));
    uint64_t nt = 0;
    if (!out->s || !get(is, nt) || nt != s->n) return false;
    out->ternary.resize(nt);
    if (!is.read(reinterpret_cast<char*>(out->ternary.data()), (std::streamsize)nt)) return false;
    sk = out;
    return true;
}

// ---- ciphertexts ----
bool Serial::Serialize(const Ciphertext<DCRTPoly>& ct, std::ostream& os, SerType::Kind k) {
    if (!binaryOnly(k) || !ct) return false;
    SfheContextState* s = unsharded(ct->cc);
    OpLock g(s);
    ct->cc->Settle(ct);  // a lazy product's rows, rescaled
    header(os, R_CT, ct->cc->Fingerprint());
    put(os, s->keyTag);
    put(os, ct->level);
    put(os, ct->slots);
    put(os, ct->scale);
    const size_t pw = s->polyWords(ct->level);
    putWords(os, s, ct->c0, pw);
    putWords(os, s, ct->c1, pw);
    return os.good();
}

bool Serial::Deserialize(Ciphertext<DCRTPoly>& ct, std::istream& is, SerType::Kind k) {
    if (!binaryOnly(k)) return false;
    uint64_t fp = 0;
    uint64_t tag = 0;
    if (!readHeader(is, R_CT, fp) || !get(is, tag)) return false;
    auto cc = findContext(fp, tag, false);
    if (!cc) {
        std::cerr << "sfhe: no live crypto context matches the ciphertext (deserialize the context first)"
                  << std::endl;
        return false;
    }
    SfheContextState* s = unsharded(cc);
    OpLock g(s);
    uint32_t level = 0, slots = 0;
    double scale = 0;
    if (!(get(is, level) && get(is, slots) && get(is, scale)) || level > s->L) return false;
    const size_t pw = s->polyWords(level);
    std::vector<uint64_t> h(2 * pw);
    for (int p = 0; p < 2; ++p) {
        uint64_t words = 0;
        if (!get(is, words) || words != pw) return false;
        if (!is.read(reinterpret_cast<char*>(h.data() + p * pw), (std::streamsize)(pw * 8))) return false;
    }
    auto out = std::make_shared<CiphertextImpl<DCRTPoly>>();
    out->cc = cc;
    out->buf = s->alloc(2 * pw);
    out->c0 = out->buf->ptr;
    out->c1 = out->c0 + pw;
    sfp_h2d(s->dev, out->c0, h.data(), 2 * pw * 8);
    s->wrote(out->buf.get());
    out->level = level;
    out->slots = slots;
    out->scale = scale;
    ct = out;
    return true;
}

// ---- evaluation keys (static, over every registered context) ----
namespace {
template <class F>
void forEachContext(F&& f) {
    std::vector<CryptoContext<DCRTPoly>> live;
    {
        std::lock_guard<std::mutex> g(g_regMu);
        for (auto& w : g_registry)
            if (auto c = w.lock()) live.push_back(c);
    }
    for (auto& c : live) f(c);
}
}  // namespace

bool CryptoContextImpl<DCRTPoly>::SerializeEvalMultKey(std::ostream& os, SerType::Kind k, const std::string& keyTag) {
    if (!binaryOnly(k)) return false;
    auto want = [&](const CryptoContext<DCRTPoly>& c) {
        return c->state()->relinKey && (keyTag.empty() || KeyTagString(c->state()->keyTag) == keyTag);
    };
    uint32_t n = 0;
    forEachContext([&](const CryptoContext<DCRTPoly>& c) { n += want(c) ? 1 : 0; });
    if (!n) return false;
    put(os, n);
    forEachContext([&](const CryptoContext<DCRTPoly>& c) {
        if (!want(c)) return;
        SfheContextState* s = unsharded(c);
        OpLock g(s);
        header(os, R_MULT, c->Fingerprint());
        put(os, s->keyTag);
        putWords(os, s, s->relinKey->ptr, s->relinKey->words);
    });
    return os.good();
}

bool CryptoContextImpl<DCRTPoly>::DeserializeEvalMultKey(std::istream& is, SerType::Kind k) {
    if (!binaryOnly(k)) return false;
    uint32_t n = 0;
    if (!get(is, n) || !n) return false;
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t fp = 0, tag = 0;
        if (!readHeader(is, R_MULT, fp) || !get(is, tag) || !tag) return false;
        auto cc = findContext(fp, tag, true);
        if (!cc) return false;
        SfheContextState* s = unsharded(cc);
        OpLock g(s);
        auto key = getWords(is, s, switchKeyWords(s));
        if (!key) return false;
        s->relinKey = key;
        s->tiersReady = false;  // (the records carry the context's keys only: switches use the whole P)
    }
    return true;
}

bool CryptoContextImpl<DCRTPoly>::SerializeEvalAutomorphismKey(std::ostream& os, SerType::Kind k,
                                                               const std::string& keyTag) {
    if (!binaryOnly(k)) return false;
    auto want = [&](const CryptoContext<DCRTPoly>& c) {
        return !c->state()->rotKeys.empty() && (keyTag.empty() || KeyTagString(c->state()->keyTag) == keyTag);
    };
    uint32_t n = 0;
    forEachContext([&](const CryptoContext<DCRTPoly>& c) { n += want(c) ? 1 : 0; });
    if (!n) return false;
    put(os, n);
    forEachContext([&](const CryptoContext<DCRTPoly>& c) {
        if (!want(c)) return;
        SfheContextState* s = unsharded(c);
        OpLock g(s);
        header(os, R_ROT, c->Fingerprint());
        put(os, s->keyTag);
        put(os, (uint32_t)s->rotKeys.size());
        for (auto& kv : s->rotKeys) {
            put(os, kv.first);
            putWords(os, s, kv.second->ptr, kv.second->words);
        }
        put(os, (uint32_t)s->rotIndices.size());
        for (int32_t r : s->rotIndices) put(os, r);
    });
    return os.good();
}

bool CryptoContextImpl<DCRTPoly>::DeserializeEvalAutomorphismKey(std::istream& is, SerType::Kind k) {
    if (!binaryOnly(k)) return false;
    uint32_t n = 0;
    if (!get(is, n) || !n) return false;
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t fp = 0, tag = 0;
        if (!readHeader(is, R_ROT, fp) || !get(is, tag) || !tag) return false;
        auto cc = findContext(fp, tag, true);
        if (!cc) return false;
        SfheContextState* s = unsharded(cc);
        OpLock g(s);
        uint32_t nk = 0, ni = 0;
        if (!get(is, nk)) return false;
        for (uint32_t j = 0; j < nk; ++j) {
            uint32_t gal = 0;
            if (!get(is, gal) || !(gal & 1) || gal >= 2 * s->n) return false;
            auto key = getWords(is, s, switchKeyWords(s));
            if (!key) return false;
            s->rotKeys[gal] = key;
            s->tiersReady = false;
        }
        if (!get(is, ni)) return false;
        for (uint32_t j = 0; j < ni; ++j) {
            int32_t r = 0;
            if (!get(is, r)) return false;
            s->rotIndices.insert(r);
        }
    }
    return true;
}

}  // namespace lbcrypto
