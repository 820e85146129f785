// RNS-CKKS context: parameters, primes, keys, encryption and the evaluator.
//
// Scheme: RNS-CKKS with HYBRID key switching (dnum digits, K special primes)
// and scale-exact automatic rescaling (FLEXIBLEAUTO-style): every ciphertext
// at level l carries the canonical scale Delta_l, with Delta_0 = 2^s and
// Delta_{l+1} = Delta_l^2 / q_{L-l}; the scaling primes are picked greedily
// so that Delta_l stays within ~2^-19 of 2^s.  Operands at different levels
// are aligned by multiplying with the integer round(Delta_t q / Delta_l) and
// rescaling, which costs no depth on the result (OpenFHE does the same).
//
// All polynomial work is enqueued through csrc/prims.h.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "state.h"

namespace lbcrypto {

// ============================================================================
// number theory helpers (host)
namespace {

u64 mulmod(u64 a, u64 b, u64 m) { return (u64)((u128)a * b % m); }
u64 powmod(u64 a, u64 e, u64 m) {
    u64 r = 1 % m;
    a %= m;
    while (e) {
        if (e & 1) r = mulmod(r, a, m);
        a = mulmod(a, a, m);
        e >>= 1;
    }
    return r;
}
u64 invmod(u64 a, u64 m) { return powmod(a % m, m - 2, m); }  // m prime

bool isPrime(u64 n) {
    if (n < 2) return false;
    static const u64 small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (u64 p : small) {
        if (n % p == 0) return n == p;
    }
    u64 d = n - 1;
    int s = 0;
    while ((d & 1) == 0) {
        d >>= 1;
        ++s;
    }
    for (u64 a : small) {
        u64 x = powmod(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int r = 1; r < s; ++r) {
            x = mulmod(x, x, n);
            if (x == n - 1) {
                comp = false;
                break;
            }
        }
        if (comp) return false;
    }
    return true;
}

// largest prime p < bound with p = 1 mod m, not in used
u64 primeBelow(u64 bound, u64 m, const std::set<u64>& used) {
    u64 c = ((bound - 1) / m) * m + 1;
    if (c >= bound) c -= m;
    for (; c > m; c -= m)
        if (!used.count(c) && isPrime(c)) return c;
    SFHE_THROW("no NTT-friendly prime found");
}

// prime p = 1 mod m closest to target, not in used
u64 primeNear(double target, u64 m, const std::set<u64>& used) {
    u64 base = (u64)std::llround((target - 1.0) / (double)m) * m + 1;
    for (u64 k = 0; k < (1u << 22); ++k) {
        u64 c1 = base + k * m;
        if (!used.count(c1) && isPrime(c1)) {
            // also look below at the same distance
            u64 c2 = base - k * m;
            if (k && c2 > m && !used.count(c2) && isPrime(c2) &&
                std::fabs((double)c2 - target) < std::fabs((double)c1 - target))
                return c2;
            return c1;
        }
        if (k) {
            u64 c2 = base - k * m;
            if (c2 > m && !used.count(c2) && isPrime(c2)) return c2;
        }
    }
    SFHE_THROW("no NTT-friendly prime near target");
}

u64 findPsi(u64 q, uint32_t n) {
    const u64 twoN = 2ull * n;
    for (u64 x = 2; x < q; ++x) {
        u64 psi = powmod(x, (q - 1) / twoN, q);
        if (powmod(psi, n, q) == q - 1) return psi;
    }
    SFHE_THROW("no primitive 2n-th root");
}

// HE-standard bound on log2(PQ) for 128-bit classical security (uniform
// ternary secret), as OpenFHE's StdLatticeParm table.
uint32_t maxLogQ128(uint32_t logn) {
    switch (logn) {
        case 10: return 27;
        case 11: return 54;
        case 12: return 109;
        case 13: return 218;
        case 14: return 438;
        case 15: return 881;
        case 16: return 1772;
        case 17: return 3524;
        default: return logn > 17 ? 7050u << (logn - 18) : 0;
    }
}

// residue of round(x) (|x| < 2^126) modulo q
u64 residueOf(double x, u64 q) {
    double r = std::nearbyint(x);
    bool neg = r < 0;
    double a = std::fabs(r);
    u128 v;
    if (a < 1.8e19) {
        v = (u128)(u64)a;
    } else {
        // split: a = hi * 2^64 + lo (exact for doubles)
        double hi = std::floor(std::ldexp(a, -64));
        double lo = a - std::ldexp(hi, 64);
        v = ((u128)(u64)hi << 64) + (u128)(u64)lo;
    }
    u64 m = (u64)(v % q);
    return neg ? (m ? q - m : 0) : m;
}

}  // namespace

// ============================================================================
// device buffers

DeviceBuffer::~DeviceBuffer() {
    if (ready) sfp_event_free(st->dev, ready);
    if (!ptr || parent) return;  // a view: the parent block returns to the pool with its last view
    std::lock_guard<std::mutex> g(st->poolMu);
    if (!st->graphOwned.empty()) {
        auto it = st->graphOwned.find(ptr);
        if (it != st->graphOwned.end()) {  // a graph addresses it: the graph releases it
            it->second = false;
            return;
        }
    }
    if (st->batchDepth && std::this_thread::get_id() == st->batchThread)
        st->batchFree.push_back({words, ptr, lane, region});  // its batch's launches are not issued yet
    else
        st->poolReturn(words, ptr, lane, region, st->myLane());
}

void SfheContextState::poolReturn(size_t words, uint64_t* p, int lane, uint64_t region, int freer) {
    if (!forkedLanes)
        freeList[0][words].push_back(p);  // everything is ordered behind lane 0 again
    else if (region == this->region && lane == freer)
        freeList[lane][words].push_back(p);  // private to this lane in this region
    else
        deferredFree.push_back({words, p});  // another lane may still use it: after the join
}

DeviceBufferPtr SfheContextState::alloc(size_t words) {
    if (!words) words = 1;  // a sharded rank may own no row of a low level
    uint64_t* p = nullptr;
    {
        std::lock_guard<std::mutex> g(poolMu);
        auto take = [&](std::map<size_t, std::vector<uint64_t*>>& fl) {
            auto it = fl.find(words);
            if (it == fl.end() || it->second.empty()) return false;
            p = it->second.back();
            it->second.pop_back();
            return true;
        };
        // own lane first; then the pre-fork pool, which every lane of a region
        // is ordered after (each waited for lane 0 at the fork)
        if (!take(freeList[lane]) && forkedLanes) take(forkPool);
    }
    if (!p) {
        p = (uint64_t*)sfp_alloc(dev, words * 8);
        if (!p) {
            // drop cached blocks and retry once
            releaseAll();
            p = (uint64_t*)sfp_alloc(dev, words * 8);
            if (!p) SFHE_THROW("device allocation failed (" + std::to_string(words * 8) + " bytes)");
        }
        poolBytes += words * 8;
    }
    auto b = std::make_shared<DeviceBuffer>(this, p, words, lane, forkedLanes ? region : 0);
    b->seq = ++laneSeq[lane];
    b->capEpoch = capturing ? captureEpoch : 0;
    if (capturing) {
        std::lock_guard<std::mutex> g(poolMu);
        capAllocs.push_back({p, words});
    }
    return b;
}

namespace {
thread_local const SfheContextState* tCtx = nullptr;
thread_local int tLane = 0;
}  // namespace

int SfheContextState::myLane() const { return tCtx == this ? tLane : 0; }
void SfheContextState::setMyLane(int l) {
    tCtx = this;
    tLane = l;
}

void SfheContextState::laneWait(int waiter, int waitee) {
    if (waiter == waitee) return;
    sfp_lane_wait(dev, waiter, waitee);
    synced[waiter][waitee] = laneSeq[waitee];
}

void SfheContextState::dep(DeviceBuffer* b) {
    if (b && b->lane != lane && synced[lane][b->lane] < b->seq) {
        static const bool stats = std::getenv("SFHE_LANE_STATS") != nullptr;
        if (stats && forkedLanes) {
            ++regionDepWaits;
            std::fprintf(stderr, "LANEWAIT lane %d waits for lane %d (buffer %zu words, seq %llu > synced %llu)\n",
                         lane, b->lane, b->words, (unsigned long long)b->seq,
                         (unsigned long long)synced[lane][b->lane]);
        }
        laneWait(lane, b->lane);
    }
}

void SfheContextState::wrote(DeviceBuffer* b) {
    b->lane = lane;
    b->seq = ++laneSeq[lane];
}

void SfheContextState::releaseAll() {
    std::lock_guard<std::mutex> g(poolMu);
    sfp_sync(dev);
    auto drop = [&](std::map<size_t, std::vector<uint64_t*>>& fl) {
        for (auto& kv : fl)
            for (auto* p : kv.second) {
                sfp_free(dev, p);
                poolBytes -= kv.first * 8;
            }
        fl.clear();
    };
    for (auto& fl : freeList) drop(fl);
    drop(forkPool);
}

// ============================================================================
// internal helpers (friend of the context)

class SfheInternal {
  public:
    using CC = CryptoContextImpl<DCRTPoly>;
    using Ct = Ciphertext<DCRTPoly>;

    // Debug: SFHE_TRACE=1 prints a hash of every op result (stderr), so the
    // traces of two backends can be diffed to find the first divergent op.
    static Ct traced(CC* cc, Ct ct, const char* what) {
        static const bool on = std::getenv("SFHE_TRACE") != nullptr;
        if (!on || ct->def) return ct;  // a deferred product is traced where it is computed
        static uint64_t counter = 0;
        SfheContextState* s = cc->st.get();
        const size_t words = s->polyWords(ct->level);
        std::vector<u64> h(words * 2);
        sfp_d2h(s->dev, h.data(), ct->c0, words * 8);
        sfp_d2h(s->dev, h.data() + words, ct->c1, words * 8);
        uint64_t f = 1469598103934665603ull;
        for (u64 v : h) f = (f ^ v) * 1099511628211ull;
        std::fprintf(stderr, "TRACE %llu %s L%u %016llx\n", (unsigned long long)counter++, what,
                     ct->level, (unsigned long long)f);
        return ct;
    }

    // Inputs in canonical form (lazy rescaling: deferred products computed,
    // pending rows rescaled), with the current lane ordered after their writers.
    static void deps(SfheContextState* s, std::initializer_list<const Ct*> in) {
        for (const Ct* c : in)
            if (c && *c) {
                materialize(**c, false);
                s->dep((*c)->buf.get());
            }
    }
    static void depsv(SfheContextState* s, const std::vector<Ct>& in) {
        for (const Ct& c : in)
            if (c) {
                materialize(*c, false);
                s->dep(c->buf.get());
            }
    }

    // ---- lazy rescaling ------------------------------------------------------
    // Products (ct x ct, ct x pt, ct x double, sums of ct x pt) return deferred
    // ciphertexts.  A consumer that can work on the product BEFORE its rescale
    // -- a rotation, or a sum with another such product or with a ciphertext
    // of a lower level (lifted exactly by an integer) -- takes the pending
    // rows; everything else takes the canonical form (the fused product +
    // rescale, as before).  Rotations of pending rows divide their key-switch
    // rounding by the prime the final rescale drops, and a sum of products is
    // rescaled once: OpenFHE's FLEXIBLEAUTO rescales lazily the same way.
    // SFHE_LAZY=0 computes every product in canonical form at once.
    static bool lazy(const SfheContextState* s) {
        static const bool on = [] {
            const char* v = std::getenv("SFHE_LAZY");
            return !v || *v != '0';
        }();
        return on && s->lazyHold == 0;
    }
    static bool isLazy(const Ct& c) { return c && (c->def || c->pend); }
    static uint32_t ctEll(const SfheContextState* s, const CiphertextImpl<DCRTPoly>& c) {
        return s->ellOf(c.level) + (c.pend ? 1u : 0u);
    }
    static void materialize(CiphertextImpl<DCRTPoly>& c, bool pendingOk) {
        if (std::shared_ptr<DeferredOp> d = takeDeferred(c, pendingOk)) d->run(c.cc.get(), c, pendingOk);
        if (c.pend && !pendingOk) settleRows(c);
    }
    // c's deferred op, taken out to be run by the caller, with the capture
    // undo record kept as materialize keeps it
    static std::shared_ptr<DeferredOp> takeDeferred(CiphertextImpl<DCRTPoly>& c, bool pendingOk) {
        SfheContextState* s = c.cc->state();
        if (c.undo && !(s->capturing && s->captureEpoch == c.undo->epoch)) {
            if (s->abandonedEpochs.count(c.undo->epoch)) {  // the capture's work never ran
                c.def = c.undo->def;
                c.buf = c.undo->buf;
                c.c0 = c.undo->c0;
                c.c1 = c.undo->c1;
                c.pend = c.undo->pend;
                c.scale = c.undo->scale;
            }
            c.undo.reset();
        }
        if (s->capturing && !c.undo && (c.def || (c.pend && !pendingOk))) {
            auto u = std::make_shared<CiphertextImpl<DCRTPoly>::CaptureUndo>();
            u->epoch = s->captureEpoch;
            u->def = c.def;
            u->buf = c.buf;
            u->c0 = c.c0;
            u->c1 = c.c1;
            u->pend = c.pend;
            u->scale = c.scale;
            c.undo = std::move(u);
        }
        std::shared_ptr<DeferredOp> d = std::move(c.def);
        c.def.reset();
        return d;
    }
    // pending rows -> their rescale (canonical, at c.level)
    static void settleRows(CiphertextImpl<DCRTPoly>& c) {
        CC* cc = c.cc.get();
        SfheContextState* s = cc->st.get();
        s->dep(c.buf.get());
        const uint32_t ell = ctEll(s, c);
        const size_t pw = s->polyWords(c.level);
        auto out = s->alloc(2 * pw);
        if (s->shardAt(ell))  // the dropped row's owner broadcasts it
            rescaleShard(s, out->ptr, c.c0, ell, 2, (size_t)(c.c1 - c.c0), pw);
        else
            sfp_rescale(s->dev, out->ptr, c.c0, ell, s->qInvTable[ell].data(), 2, (size_t)(c.c1 - c.c0), pw);
        s->stats.rescale++;
        s->countBytes(4.0 * ell * s->n * 8);
        c.buf = out;
        c.c0 = out->ptr;
        c.c1 = out->ptr + pw;
        c.pend = false;
        c.scale = s->scale[c.level];
    }
    // a deferred result at post-rescale `level`
    static Ct deferredCt(CC* cc, uint32_t level, uint32_t slots, std::shared_ptr<DeferredOp> op) {
        SfheContextState* s = cc->st.get();
        auto ct = std::make_shared<CiphertextImpl<DCRTPoly>>();
        ct->cc = cc->shared_from_this();
        ct->level = level;
        ct->slots = slots;
        ct->scale = s->scale[level];
        ct->def = std::move(op);
        return ct;
    }
    // a fresh pending ciphertext: rows for ellOf(level) + 1 limbs
    static Ct newPendingCt(CC* cc, uint32_t level, uint32_t slots) {
        SfheContextState* s = cc->st.get();
        auto ct = std::make_shared<CiphertextImpl<DCRTPoly>>();
        const size_t pw = s->polyWords(level - 1);
        ct->cc = cc->shared_from_this();
        ct->buf = s->alloc(2 * pw);
        ct->c0 = ct->buf->ptr;
        ct->c1 = ct->c0 + pw;
        ct->level = level;
        ct->slots = slots;
        ct->scale = s->preScale(level);
        ct->pend = true;
        return ct;
    }
    // Sum / difference of two ciphertexts where at least one is a lazy
    // product: null if the canonical path must be taken instead.  The result
    // is pending at their common level; a canonical operand of a lower level
    // is lifted onto the product's scale by an integer multiple (exact up to
    // a relative 2^-41 of its value -- no rounding noise).
    static Ct lazyAdd(CC* cc, const Ct& a, const Ct& b, bool sub) {
        SfheContextState* s = cc->st.get();
        if (!lazy(s) || !(isLazy(a) || isLazy(b))) return nullptr;
        const Ct* lz[2] = {&a, &b};
        bool liftIdx[2] = {false, false};
        if (isLazy(a) && isLazy(b)) {
            if (a->level != b->level) return nullptr;
        } else {
            const Ct& c = isLazy(a) ? b : a;   // the canonical one
            const Ct& p = isLazy(a) ? a : b;
            if (c->level >= p->level) return nullptr;
            liftIdx[isLazy(a) ? 1 : 0] = true;
        }
        const uint32_t level = a->level > b->level ? a->level : b->level;
        for (int i = 0; i < 2; ++i) {
            materialize(**lz[i], !liftIdx[i]);
            s->dep((*lz[i])->buf.get());
        }
        const uint32_t ell = s->ellOf(level) + 1;
        const sfp_limbs m = s->qmap(ell);
        Ct out = newPendingCt(cc, level, std::max(a->slots, b->slots));
        // out = w_0 x_0 + w_1 x_1 for both polynomials in one launch: w = 1,
        // or the lift's integer for a canonical operand; -w for a subtrahend
        const uint64_t* x0[2];
        const uint64_t* x1[2];
        std::vector<u64> w(2 * (size_t)m.count);
        DeviceBufferPtr gathered;  // a sharded operand read at a replicated (tail) limb count
        for (int i = 0; i < 2; ++i) {
            const Ct& c = *lz[i];
            x0[i] = c->c0;
            x1[i] = c->c1;
            if (liftIdx[i] && s->shardAt(s->ellOf(c->level)) && !s->shardAt(ell)) {
                gathered = gatherRows(s, c->c0, c->c1, ell);
                x0[i] = gathered->ptr;
                x1[i] = gathered->ptr + (size_t)ell * s->n;
            }
            const std::vector<u64> k = liftIdx[i] ? constResidues(s, s->preScale(level) / c->scale, ell)
                                                  : std::vector<u64>(m.count, 1);
            for (uint32_t r = 0; r < m.count; ++r) {
                const u64 q = s->primes[s->qprime(r, ell)];
                w[(size_t)i * m.count + r] = (sub && i == 1) ? (k[r] ? q - k[r] : 0) : k[r];
            }
        }
        sfp_lin_wsum_multi(s->dev, out->c0, 0, (size_t)(out->c1 - out->c0), x0, x1, 2, w.data(), 1, m);
        s->stats.add++;
        s->countBytes(6.0 * ell * s->n * 8);
        return out;
    }

    static sfp_limbs Q(uint32_t ell) { return sfp_limbs{ell, ell, 0}; }
    // both polynomials of ciphertexts laid out [c0 rows][c1 rows] in one launch:
    // rows [r, 2r) repeat the primes of rows [0, r)
    static bool packed(const SfheContextState* s, std::initializer_list<const uint64_t*> c0s,
                       std::initializer_list<const uint64_t*> c1s, uint32_t level) {
        const size_t pw = s->polyWords(level);
        auto a = c0s.begin();
        for (auto b = c1s.begin(); b != c1s.end(); ++a, ++b)
            if (*b != *a + pw) return false;
        return true;
    }
    static sfp_limbs both(const SfheContextState* s, uint32_t ell) {
        sfp_limbs m = s->qmap(ell);
        m.count *= 2;
        m.pbase = m.base;
        return m;
    }
    static sfp_limbs Range(uint32_t lo, uint32_t cnt) { return sfp_limbs{cnt, 0, lo}; }

    static Ct newCt(CC* cc, uint32_t level, uint32_t slots) {
        SfheContextState* s = cc->st.get();
        auto ct = std::make_shared<CiphertextImpl<DCRTPoly>>();
        const size_t pw = s->polyWords(level);
        ct->cc = cc->shared_from_this();
        ct->buf = s->alloc(2 * pw);
        ct->c0 = ct->buf->ptr;
        ct->c1 = ct->c0 + pw;
        ct->level = level;
        ct->slots = slots;
        ct->scale = s->scale[level];
        return ct;
    }

    // residues of round(v) modulo the primes of the local rows of ell limbs
    static std::vector<u64> constResidues(SfheContextState* s, double v, uint32_t ell) {
        std::vector<u64> k(s->rows(ell));
        for (uint32_t i = 0; i < k.size(); ++i) k[i] = residueOf(v, s->primes[s->qprime(i, ell)]);
        return k;
    }

    // (c0,c1) at level l, ell limbs, any scale -> new ct at level l+1
    static Ct rescale(CC* cc, const uint64_t* c0, const uint64_t* c1, uint32_t level,
                      uint32_t slots) {
        SfheContextState* s = cc->st.get();
        uint32_t ell = s->ellOf(level);
        if (ell < 2) SFHE_THROW("no levels left to rescale (multiplicative depth exhausted)");
        Ct out = newCt(cc, level + 1, slots);
        if (c1 - c0 < 0) SFHE_THROW("internal: layout");
        if (s->shardAt(ell))
            rescaleShard(s, out->c0, c0, ell, 2, (size_t)(c1 - c0), (size_t)(out->c1 - out->c0));
        else
            sfp_rescale(s->dev, out->c0, c0, ell, s->qInvTable[ell].data(), 2, (size_t)(c1 - c0),
                        (size_t)(out->c1 - out->c0));
        s->stats.rescale++;
        s->countBytes(4.0 * ell * s->n * 8 * 2 / 2);  // 4 l B per poly pair
        return out;
    }

    // Align ct to targetLevel (>= its level) with a scale-exact adjustment;
    // factor != 1 also multiplies the values by factor (same constant).
    static Ct adjust(CC* cc, const Ct& ct, uint32_t target, double factor = 1.0) {
        SfheContextState* s = cc->st.get();
        if (target == ct->level && factor == 1.0) return ct;
        if (target <= ct->level && factor != 1.0) SFHE_THROW("a scaled adjustment needs a level to consume");
        if (target < ct->level) SFHE_THROW("cannot raise a ciphertext's level");
        if (target > s->L) SFHE_THROW("target level beyond multiplicative depth");
        uint32_t mid = target - 1;  // drop limbs (free), then one scaled rescale
        uint32_t ell = s->ellOf(mid);
        // result scale = scale_ct * K / q_{ell-1} = Delta_target
        double K = factor * s->scale[target] * (double)s->primes[ell - 1] / ct->scale;
        auto k = constResidues(s, K, ell);
        s->stats.constmult++;
        s->countBytes(4.0 * ell * s->n * 8);
        if (s->shardAt(s->ellOf(ct->level)) && !s->shardAt(ell)) {
            // from dealt rows into the replicated tail: every row of the kept limbs first
            auto full = gatherRows(s, ct->c0, ct->c1, ell);
            auto v = view(cc, full, full->ptr, full->ptr + (size_t)ell * s->n, ct->level, ct->scale, ct->slots);
            return mulRescale(cc, v, mid, k.data(), nullptr, ct->slots);
        }
        return mulRescale(cc, ct, mid, k.data(), nullptr, ct->slots);
    }

    // SFHE_FUSED_RESCALE=0 selects the two-step paths (product, then rescale)
    // the fused prims replace; tests check both agree bit for bit.
    static bool fusedRescale() {
        static const bool on = [] {
            const char* v = std::getenv("SFHE_FUSED_RESCALE");
            return !v || *v != '0';
        }();
        return on;
    }

    // Rescale(ct * k) (k: ell per-row residues) or Rescale(ct (.) m) (m: ell
    // plaintext rows) in one fused prim; ct's first ellOf(level) rows are used.
    static Ct mulRescale(CC* cc, const Ct& ct, uint32_t level, const u64* k, const uint64_t* m,
                         uint32_t slots) {
        SfheContextState* s = cc->st.get();
        const uint32_t ell = s->ellOf(level);
        if (ell < 2) SFHE_THROW("no levels left to rescale (multiplicative depth exhausted)");
        if (!fusedRescale() || s->shardAt(ell)) {
            const size_t pw = s->polyWords(level);
            auto tmp = s->alloc(2 * pw);
            uint64_t* t0 = tmp->ptr;
            uint64_t* t1 = t0 + pw;
            if (k) {
                sfp_mul_const(s->dev, t0, ct->c0, k, s->qmap(ell));
                sfp_mul_const(s->dev, t1, ct->c1, k, s->qmap(ell));
            } else {
                sfp_mul(s->dev, t0, ct->c0, m, s->qmap(ell));
                sfp_mul(s->dev, t1, ct->c1, m, s->qmap(ell));
            }
            return rescale(cc, t0, t1, level, slots);
        }
        Ct out = newCt(cc, level + 1, slots);
        const size_t inStride = (size_t)(ct->c1 - ct->c0), outStride = (size_t)(out->c1 - out->c0);
        if (k)
            sfp_mul_const_rescale(s->dev, out->c0, ct->c0, k, ell, s->qInvTable[ell].data(), 2, inStride,
                                  outStride);
        else
            sfp_mul_rescale(s->dev, out->c0, ct->c0, m, ell, s->qInvTable[ell].data(), 2, inStride,
                            outStride);
        s->stats.rescale++;
        s->countBytes(4.0 * ell * s->n * 8 * 2 / 2);
        return out;
    }

    static void align(CC* cc, Ct& a, Ct& b) {
        uint32_t l = std::max(a->level, b->level);
        a = adjust(cc, a, l);
        b = adjust(cc, b, l);
    }

    // ---- limb sharding: this rank computes its own rows; the
    // exchange steps are the ModUp input (all Q rows, coefficient form), the
    // ModDown P rows and the dropped row of a rescale.  Row order of a
    // gathered buffer: rank-major blocks of `per` rows (rank r's local row i
    // at r * per + i), i.e. global row g at (g % W) * per + g / W.
    static std::vector<uint32_t> naturalOrder(const SfheContextState* s, uint32_t count, uint32_t per,
                                              uint32_t blocks = 1, uint32_t block = 0) {
        std::vector<uint32_t> r(count);
        for (uint32_t g = 0; g < count; ++g)
            r[g] = ((g % s->world) * blocks + block) * per + g / s->world;
        return r;
    }

    // Every row of the first `ell` limbs of a ciphertext dealt over the ranks
    // (c0 / c1: its local rows, a prefix of which are those limbs'), in
    // natural order on every rank: 2 * ell rows, c0 then c1.  One all-gather.
    static DeviceBufferPtr gatherRows(SfheContextState* s, const uint64_t* c0, const uint64_t* c1, uint32_t ell) {
        const uint32_t n = s->n, lr = s->owned(ell);
        const uint32_t per = (ell + s->world - 1) / s->world;
        auto send = s->alloc((size_t)2 * per * n);
        if (lr) {
            sfp_d2d(s->dev, send->ptr, c0, (size_t)lr * n * 8);
            sfp_d2d(s->dev, send->ptr + (size_t)per * n, c1, (size_t)lr * n * 8);
        }
        auto all = s->alloc((size_t)2 * per * s->world * n);
        sfp_allgather(s->dev, send->ptr, all->ptr, (size_t)2 * per * n * 8);
        auto full = s->alloc((size_t)2 * ell * n);
        for (uint32_t p = 0; p < 2; ++p) {
            auto idx = naturalOrder(s, ell, per, 2, p);
            sfp_gather_rows(s->dev, full->ptr + (size_t)p * ell * n, all->ptr, idx.data(), ell);
        }
        return full;
    }

    // coefficient-form rows of every limb of `local` (this rank's dealt rows
    // of ell limbs, evaluation domain) in natural order into `nat` (ell rows)
    static void gatherCoeff(SfheContextState* s, uint64_t* nat, const uint64_t* local, uint32_t ell) {
        const uint32_t n = s->n, per = (ell + s->world - 1) / s->world, lr = s->owned(ell);
        auto send = s->alloc((size_t)per * n);
        auto all = s->alloc((size_t)per * s->world * n);
        if (lr) {
            sfp_d2d(s->dev, send->ptr, local, (size_t)lr * n * 8);
            sfp_ntt(s->dev, send->ptr, s->shardMap(ell), 1);
        }
        sfp_allgather(s->dev, send->ptr, all->ptr, (size_t)per * n * 8);
        auto idx = naturalOrder(s, ell, per);
        sfp_gather_rows(s->dev, nat, all->ptr, idx.data(), ell);
    }

    // conversion tables with this rank's targets: ModUp digit j of ell limbs
    // -> every local ext row (own-digit rows included: the conversion of a
    // row to its own prime returns it exactly)
    static std::vector<sfp_conv*>& modupConvShard(SfheContextState* s, uint32_t ell) {
        auto it = s->modupConvShard.find(ell);
        if (it != s->modupConvShard.end()) return it->second;
        std::vector<sfp_conv*> v;
        const uint32_t beta = (ell + s->alpha - 1) / s->alpha;
        std::vector<uint32_t> dst;
        for (uint32_t i = 0; i < s->owned(ell); ++i) dst.push_back(s->qprimeShard(i));
        for (uint32_t k = 0; k < s->owned(s->K); ++k) dst.push_back(s->Lq + s->rank + k * s->world);
        for (uint32_t j = 0; j < beta; ++j) {
            std::vector<uint32_t> src;
            for (uint32_t i = j * s->alpha; i < std::min((j + 1) * s->alpha, ell); ++i) src.push_back(i);
            v.push_back(makeConv(s, src, dst));
        }
        return s->modupConvShard[ell] = v;
    }

    // This rank's slice of a whole switching key (sfp_key_geom): per digit
    // and part, the tail Q rows, the rank's dealt Q rows above the tail and
    // the P rows -- every row a replicated level or this rank's dealt rows
    // read.
    // A tier's key (one digit over Lq + K' rows) takes the same layout: its
    // K' P rows at pstart.., the slots of the P primes it lacks zero.
    static DeviceBufferPtr sliceKey(SfheContextState* s, const DeviceBufferPtr& whole, int tier = -1) {
        const sfp_key_geom& g = s->kgeom;
        const uint32_t n = s->n, NP = s->Lq + s->Kof(tier), digits = tier < 0 ? s->dnum : 1;
        std::vector<uint32_t> rows;
        for (uint32_t p = 0; p < s->Lq + s->K; ++p) {
            const bool keep = p < g.tail || p >= s->Lq || p % g.world == (uint32_t)s->rank;
            if (!keep) continue;
            if (sfp_key_row(&g, p) != rows.size()) SFHE_THROW("internal: key slice row map");
            rows.push_back(p);
        }
        if (rows.size() != g.rows) SFHE_THROW("internal: key slice size");
        auto out = s->alloc((size_t)digits * 2 * g.rows * n);
        out->ksTier = tier;
        const uint32_t have = NP < s->Lq + s->K ? g.pstart + (NP - s->Lq) : g.rows;  // rows a tier key fills
        for (uint32_t part = 0; part < 2 * digits; ++part) {
            uint64_t* o = out->ptr + (size_t)part * g.rows * n;
            sfp_gather_rows(s->dev, o, whole->ptr + (size_t)part * NP * n, rows.data(), have);
            if (have < g.rows) sfp_zero(s->dev, o + (size_t)have * n, (size_t)(g.rows - have) * n * 8);
        }
        return out;
    }

    // modupConvShard split for the overlapped ModUp: per digit (own rows'
    // part, the rest's part); the own rows of digit j are local rows
    // ceil((j alpha - rank) / W) .. in this rank's coefficient buffer
    static std::vector<std::pair<sfp_conv*, sfp_conv*>>& modupConvSplit(SfheContextState* s, uint32_t ell) {
        auto it = s->modupConvSplit.find(ell);
        if (it != s->modupConvSplit.end()) return it->second;
        std::vector<std::pair<sfp_conv*, sfp_conv*>> v;
        const uint32_t beta = (ell + s->alpha - 1) / s->alpha;
        std::vector<uint32_t> dst;
        for (uint32_t i = 0; i < s->owned(ell); ++i) dst.push_back(s->qprimeShard(i));
        for (uint32_t k = 0; k < s->owned(s->K); ++k) dst.push_back(s->Lq + s->rank + k * s->world);
        for (uint32_t j = 0; j < beta; ++j) {
            std::vector<uint32_t> src;
            std::vector<char> own, rest;
            for (uint32_t i = j * s->alpha; i < std::min((j + 1) * s->alpha, ell); ++i) {
                src.push_back(i);
                own.push_back(i % s->world == (uint32_t)s->rank);
                rest.push_back(!own.back());
            }
            const bool any = std::find(own.begin(), own.end(), 1) != own.end();
            v.push_back({any ? makeConv(s, src, dst, nullptr, &own, false) : nullptr,
                         makeConv(s, src, dst, nullptr, &rest, true)});
        }
        return s->modupConvSplit[ell] = v;
    }

    // The overlapped ModUp (SFHE_SHARD_OVERLAP, on by default): the all-gather
    // of the coefficient rows runs on a lane of its own while this lane
    // converts the rank's OWN rows of every digit (they need no exchange);
    // then the rest's part is added (the parts sum mod each target prime to
    // the whole conversion: the same residues) and the NTT runs.  Without a
    // spare lane (the oracle's single synchronous lane, a region using every
    // lane) the same split runs in order on this lane.  Returns false with
    // SFHE_SHARD_OVERLAP=0 (the caller runs the unsplit form).
    static bool modupShardOverlap(SfheContextState* s, uint64_t* ext, const uint64_t* d, uint32_t ell) {
        static const bool on = [] {
            const char* v = std::getenv("SFHE_SHARD_OVERLAP");
            return !v || *v != '0';
        }();
        if (!on) return false;
        const int L = sfp_get_lane(s->dev), C0 = sfp_lanes(s->dev) - 1;
        const int C = (C0 > L && C0 >= std::max(1, s->forkedLanes)) ? C0 : L;
        const uint32_t n = s->n, beta = (ell + s->alpha - 1) / s->alpha, W = (uint32_t)s->world;
        const uint32_t per = (ell + W - 1) / W, lr = s->owned(ell);
        const sfp_limbs em = s->extmap(ell);
        const size_t stride = (size_t)em.count * n;
        auto& parts = modupConvSplit(s, ell);
        auto send = s->alloc((size_t)per * n);
        auto all = s->alloc((size_t)per * W * n);
        auto nat = s->alloc((size_t)ell * n);
        auto tmp = s->alloc(stride);
        if (lr) {
            sfp_d2d(s->dev, send->ptr, d, (size_t)lr * n * 8);
            sfp_ntt(s->dev, send->ptr, s->shardMap(ell), 1);
        }
        // the exchange on lane C, after this lane's INTT
        if (C != L) {
            sfp_lane_wait(s->dev, C, L);
            sfp_set_lane(s->dev, C);
        }
        sfp_allgather(s->dev, send->ptr, all->ptr, (size_t)per * n * 8);
        auto idx = naturalOrder(s, ell, per);
        sfp_gather_rows(s->dev, nat->ptr, all->ptr, idx.data(), ell);
        sfp_set_lane(s->dev, L);
        // meanwhile: every digit's conversion of this rank's own rows
        for (uint32_t j = 0; j < beta; ++j) {
            uint64_t* e = ext + j * stride;
            const uint32_t lo = j * s->alpha;
            const uint32_t first = (lo + W - 1 - (uint32_t)s->rank) / W;  // local index of its first own row
            if (parts[j].first)
                sfp_conv_apply(s->dev, e, send->ptr + (size_t)first * n, parts[j].first);
            else
                sfp_zero(s->dev, e, stride * 8);
        }
        // the rest's part once the rows arrived, then the NTT
        if (C != L) sfp_lane_wait(s->dev, L, C);
        for (uint32_t j = 0; j < beta; ++j) {
            uint64_t* e = ext + j * stride;
            sfp_conv_apply(s->dev, tmp->ptr, nat->ptr + (size_t)j * s->alpha * n, parts[j].second);
            sfp_add(s->dev, e, e, tmp->ptr, em);
            sfp_ntt(s->dev, e, em, 0);
        }
        return true;
    }

    // ModUp of the local rows of d (ell limbs, dealt): beta blocks of extmap(ell) rows
    static void modupShard(SfheContextState* s, uint64_t* ext, const uint64_t* d, uint32_t ell) {
        if (modupShardOverlap(s, ext, d, ell)) return;
        const uint32_t n = s->n, beta = (ell + s->alpha - 1) / s->alpha;
        const sfp_limbs em = s->extmap(ell);
        const size_t stride = (size_t)em.count * n;
        auto nat = s->alloc((size_t)ell * n);
        gatherCoeff(s, nat->ptr, d, ell);
        auto& convs = modupConvShard(s, ell);
        for (uint32_t j = 0; j < beta; ++j) {
            sfp_conv_apply(s->dev, ext + j * stride, nat->ptr + (size_t)j * s->alpha * n, convs[j]);
            sfp_ntt(s->dev, ext + j * stride, em, 0);
        }
    }

    // inner product with the local key rows + ModDown to the local Q rows
    static void innerModDownShard(SfheContextState* s, const uint64_t* ext, size_t stride, uint32_t beta,
                                  uint32_t ell, const DeviceBufferPtr& key, uint64_t* out0, uint64_t* out1,
                                  int add0, int add1) {
        const size_t aw = (size_t)s->extmap(ell).count * s->n;
        auto acc = s->alloc(2 * aw);
        innerShard(s, acc->ptr, ext, stride, beta, ell, key, 0);
        modDownShard(s, acc->ptr, ell, out0, out1, add0, add1);
    }
    // The local key inner product into acc (2 polys of extmap(ell) rows),
    // accumulated when accum.  A local ext row reads the key row of its own
    // prime (sfp_key_row: in this rank's key slice).
    static void innerShard(SfheContextState* s, uint64_t* acc, const uint64_t* ext, size_t stride, uint32_t beta,
                           uint32_t ell, const DeviceBufferPtr& key, int accum) {
        const sfp_limbs em = s->extmap(ell);
        const size_t aw = (size_t)em.count * s->n;
        sfp_ks_inner_map(s->dev, acc, acc + aw, ext, stride, key->ptr, beta, em, SFP_KEY_ROW_BY_PRIME,
                         s->keyRows(), accum);
    }
    // ModDown of the local accumulators (their P rows are destroyed)
    static void modDownShard(SfheContextState* s, uint64_t* acc, uint32_t ell, uint64_t* out0, uint64_t* out1,
                             int add0, int add1) {
        const uint32_t n = s->n, K = s->K, lr = s->owned(ell), lp = s->owned(K);
        const size_t aw = (size_t)s->extmap(ell).count * n;
        // P rows: coefficient form, exchanged (both polys in one all-gather)
        const uint32_t per = (K + s->world - 1) / s->world;
        auto send = s->alloc((size_t)2 * per * n);
        const sfp_limbs pm{lp, 0, s->Lq + (uint32_t)s->rank, 0, (uint32_t)s->world};
        for (int p = 0; p < 2; ++p) {
            if (!lp) break;
            uint64_t* dst = send->ptr + (size_t)p * per * n;
            sfp_d2d(s->dev, dst, acc + p * aw + (size_t)lr * n, (size_t)lp * n * 8);
            sfp_ntt(s->dev, dst, pm, 1);
        }
        auto all = s->alloc((size_t)2 * per * s->world * n);
        sfp_allgather(s->dev, send->ptr, all->ptr, (size_t)2 * per * n * 8);
        auto natP = s->alloc((size_t)2 * K * n);
        for (uint32_t p = 0; p < 2; ++p) {
            auto idx = naturalOrder(s, K, per, 2, p);
            sfp_gather_rows(s->dev, natP->ptr + (size_t)p * K * n, all->ptr, idx.data(), K);
        }
        if (!lr) return;
        // (acc_Q - NTT(Conv_centred(P rows))) * P^-1  (+ out)
        std::vector<u64> pinv(lr);
        for (uint32_t i = 0; i < lr; ++i) pinv[i] = s->pInvModQ[s->qprimeShard(i)];
        auto conv = s->alloc((size_t)lr * n);
        uint64_t* outs[2] = {out0, out1};
        const int adds[2] = {add0, add1};
        const sfp_limbs qm = s->shardMap(ell);
        for (int p = 0; p < 2; ++p) {
            sfp_conv_apply_centered(s->dev, conv->ptr, natP->ptr + (size_t)p * K * n, s->moddownConvShard, lr);
            sfp_ntt(s->dev, conv->ptr, qm, 0);
            sfp_sub(s->dev, conv->ptr, acc + p * aw, conv->ptr, qm);
            sfp_mul_const(s->dev, conv->ptr, conv->ptr, pinv.data(), qm);
            if (adds[p])
                sfp_add(s->dev, outs[p], outs[p], conv->ptr, qm);
            else
                sfp_d2d(s->dev, outs[p], conv->ptr, (size_t)lr * n * 8);
        }
    }

    static void keySwitchShard(CC* cc, const uint64_t* d, uint32_t ell, const DeviceBufferPtr& key,
                               uint64_t* out0, uint64_t* out1, int add0, int add1) {
        SfheContextState* s = cc->st.get();
        const uint32_t beta = (ell + s->alpha - 1) / s->alpha;
        const size_t stride = (size_t)s->extmap(ell).count * s->n;
        auto ext = s->alloc(stride * beta);
        modupShard(s, ext->ptr, d, ell);
        innerModDownShard(s, ext->ptr, stride, beta, ell, key, out0, out1, add0, add1);
        s->stats.keyswitch++;
        s->countBytes((3.0 * ell + 2.0 * beta * (ell + s->K)) * s->n * 8);
    }

    // Rescale of npoly polys (this rank's dealt rows of ell limbs) by
    // q_{ell-1}: its owner broadcasts the dropped row in coefficient form.
    // When ell - 1 limbs fall in the replicated tail every rank then gathers
    // every row of the result (out: ell - 1 rows per poly).
    static void rescaleShard(SfheContextState* s, uint64_t* out, const uint64_t* in, uint32_t ell, uint32_t npoly,
                             size_t inStride, size_t outStride) {
        const uint32_t n = s->n, drop = ell - 1, owner = drop % s->world;
        auto last = s->alloc((size_t)npoly * n);
        if ((uint32_t)s->rank == owner) {
            const uint32_t lr = s->owned(ell);
            for (uint32_t p = 0; p < npoly; ++p)
                sfp_d2d(s->dev, last->ptr + (size_t)p * n, in + p * inStride + (size_t)(lr - 1) * n, (size_t)n * 8);
            for (uint32_t p = 0; p < npoly; ++p)
                sfp_ntt(s->dev, last->ptr + (size_t)p * n, sfp_limbs{1, 1, 0, drop, 1}, 1);
        }
        sfp_bcast(s->dev, last->ptr, (size_t)npoly * n * 8, (int)owner);
        const uint32_t lo = s->owned(ell - 1);
        std::vector<u64> qlinv(lo);
        for (uint32_t i = 0; i < lo; ++i) qlinv[i] = s->qInvTable[ell][s->qprimeShard(i)];
        if (s->shardAt(ell - 1)) {
            sfp_rescale_rows(s->dev, out, in, last->ptr, drop, s->shardMap(ell - 1), qlinv.data(), npoly, inStride,
                             outStride, n);
            return;
        }
        // into the replicated tail: this rank's rows of the result, then an all-gather
        const uint32_t per = (ell - 1 + s->world - 1) / s->world;
        auto mine = s->alloc((size_t)npoly * per * n);
        sfp_rescale_rows(s->dev, mine->ptr, in, last->ptr, drop, s->shardMap(ell - 1), qlinv.data(), npoly, inStride,
                         (size_t)per * n, n);
        auto all = s->alloc((size_t)npoly * per * s->world * n);
        sfp_allgather(s->dev, mine->ptr, all->ptr, (size_t)npoly * per * n * 8);
        for (uint32_t p = 0; p < npoly; ++p) {
            auto idx = naturalOrder(s, ell - 1, per, npoly, p);
            sfp_gather_rows(s->dev, out + p * outStride, all->ptr, idx.data(), ell - 1);
        }
    }

    // this rank's rows of a ciphertext computed on every row (FullScope)
    static Ct localize(CC* cc, const Ct& full) {
        SfheContextState* s = cc->st.get();
        const uint32_t ell = s->ellOf(full->level);
        if (!s->shardAt(ell)) return full;
        const uint32_t lr = s->rows(ell);
        Ct out = newCt(cc, full->level, full->slots);
        out->scale = full->scale;
        std::vector<uint32_t> idx(lr);
        for (uint32_t i = 0; i < lr; ++i) idx[i] = s->qprimeShard(i);
        sfp_gather_rows(s->dev, out->c0, full->c0, idx.data(), lr);
        sfp_gather_rows(s->dev, out->c1, full->c1, idx.data(), lr);
        return out;
    }

    // every row of a ciphertext in natural order (2 * ell rows: c0 then c1),
    // on every rank (a collective when its rows are dealt)
    static DeviceBufferPtr gatherFull(SfheContextState* s, const Ct& a) {
        const uint32_t ell = s->ellOf(a->level);
        if (s->shardAt(ell)) return gatherRows(s, a->c0, a->c1, ell);
        auto full = s->alloc((size_t)2 * ell * s->n);
        sfp_d2d(s->dev, full->ptr, a->c0, (size_t)ell * s->n * 8);
        sfp_d2d(s->dev, full->ptr + (size_t)ell * s->n, a->c1, (size_t)ell * s->n * 8);
        return full;
    }

    // ModUp of d (ell limbs, evaluation domain, unsharded rows) and the key
    // inner product into acc (two polys of ell+K rows, (ell+K)*n apart):
    // accumulated when accum, + foldK * (fold0, fold1) on row ell-1 when
    // fold0.  One fused pass where the backend has it (sfp_modup_inner: the
    // extended digits never round-trip through HBM), else ModUp + inner
    // product.  invFrom: rows t >= invFrom may leave after the first pass of
    // the ModDown's inverse NTT; returns whether they did (the ModDown's
    // row_done).
    static int modupInner(CC* cc, uint64_t* acc, const uint64_t* d, uint32_t ell, const DeviceBufferPtr& key,
                          const uint64_t* fold0, const uint64_t* fold1, u64 foldK, int accum,
                          uint32_t invFrom = ~0u) {
        SfheContextState* s = cc->st.get();
        const uint32_t n = s->n, K = s->Kof(key->ksTier);  // (the key's special-prime tier)
        const uint32_t beta = (ell + s->alpha - 1) / s->alpha;
        const size_t stride = (size_t)(ell + K) * n;
        auto ext = s->alloc(stride * beta);
        auto scratch = s->alloc((size_t)ell * n);
        auto& convs = modupConv(cc, ell, key->ksTier);
        if (sfp_modup_inner(s->dev, acc, acc + stride, d, ell, K, s->Lq, s->alpha, convs.data(), key->ptr, fold0,
                            fold1, foldK, accum, invFrom, ext->ptr, scratch->ptr) == 0)
            return invFrom != ~0u;
        sfp_modup(s->dev, ext->ptr, d, ell, K, s->Lq, s->alpha, convs.data(), scratch->ptr);
        if (fold0)
            sfp_ks_inner_fold(s->dev, acc, acc + stride, ext->ptr, stride, key->ptr, beta, ell, K, s->Lq, fold0, fold1,
                              foldK);
        else
            (accum ? sfp_ks_inner_acc : sfp_ks_inner)(s->dev, acc, acc + stride, ext->ptr, stride, key->ptr, beta,
                                                       ell, K, s->Lq);
        return 0;
    }

    // Hybrid key switch of d (ell limbs, evaluation domain) with `key`; the
    // result goes to (out0, out1) (ell limbs each), added when add0 / add1.
    static void keySwitch(CC* cc, const uint64_t* d, uint32_t ell, const DeviceBufferPtr& key,
                          uint64_t* out0, uint64_t* out1, int add0, int add1) {
        SfheContextState* s = cc->st.get();
        if (s->shardAt(ell)) return keySwitchShard(cc, d, ell, key, out0, out1, add0, add1);
        const int tier = key->ksTier;
        const uint32_t n = s->n, K = s->Kof(tier);
        const uint32_t beta = (ell + s->alpha - 1) / s->alpha;
        const size_t stride = (size_t)(ell + K) * n;
        auto acc = s->alloc(2 * stride);
        const int rowDone = modupInner(cc, acc->ptr, d, ell, key, nullptr, nullptr, 0, 0, ell);
        auto md = s->alloc((size_t)2 * ell * n);
        sfp_moddown2(s->dev, out0, out1, acc->ptr, stride, ell, K, s->Lq, s->moddownConvOf(tier), s->pInvModQof(tier),
                     add0, add1, md->ptr, rowDone);
        s->stats.keyswitch++;
        // (3 l + 2 beta (l+K)) B
        s->countBytes((3.0 * ell + 2.0 * beta * (ell + K)) * n * 8);
    }

    // EvalMult's tail: relinearise (d0, d1, d2) at `level` and rescale, with the
    // ModDown and the rescale fused (sfp_moddown_rescale): the same result as
    // keySwitch(d2, +d0, +d1) followed by rescale(), four launches fewer.
    static Ct relinRescale(CC* cc, uint64_t* d0, uint64_t* d1, const uint64_t* d2, uint32_t level,
                           uint32_t slots) {
        SfheContextState* s = cc->st.get();
        const uint32_t ell = s->ellOf(level);
        if (ell < 2) SFHE_THROW("no levels left to rescale (multiplicative depth exhausted)");
        if (s->shardAt(ell)) {
            keySwitchShard(cc, d2, ell, s->relinKey, d0, d1, 1, 1);
            return rescale(cc, d0, d1, level, slots);
        }
        const DeviceBufferPtr& key = s->relinFor(ell);
        const int tier = key->ksTier;
        const uint32_t n = s->n, K = s->Kof(tier);
        const uint32_t beta = (ell + s->alpha - 1) / s->alpha;
        const size_t stride = (size_t)(ell + K) * n;
        auto acc = s->alloc(2 * stride);
        const int rowDone = modupInner(cc, acc->ptr, d2, ell, key, d0, d1, s->pModQof(tier)[ell - 1], 0, ell - 1);
        Ct out = newCt(cc, level + 1, slots);
        auto scratch = s->alloc((size_t)2 * (ell - 1) * n);
        sfp_moddown_rescale(s->dev, out->c0, out->c1, d0, d1, acc->ptr, stride, ell, K, s->Lq,
                            s->moddownConvOf(tier), s->pInvModQof(tier), s->pModQof(tier),
                            s->qInvTable[ell].data(), scratch->ptr, rowDone);
        s->stats.keyswitch++;
        s->stats.rescale++;
        s->countBytes((3.0 * ell + 2.0 * beta * (ell + K)) * n * 8);
        s->countBytes(4.0 * ell * n * 8);
        return out;
    }

    // EvalMult(ct, ct)'s whole canonical tail from the aligned operands
    // (a0, a1), (b0, b1) at `level`: one fused pass chain where the backend
    // has it (sfp_mult_relin_rescale: the tensor is formed inside the key
    // switch's passes, never written out), else the tensor then relinRescale.
    static Ct multRelinRescale(CC* cc, const uint64_t* a0, const uint64_t* a1, const uint64_t* b0,
                               const uint64_t* b1, uint32_t level, uint32_t slots) {
        SfheContextState* s = cc->st.get();
        const uint32_t ell = s->ellOf(level);
        if (ell < 2) SFHE_THROW("no levels left to rescale (multiplicative depth exhausted)");
        const size_t pw = s->polyWords(level);
        if (!s->shardAt(ell)) {
            const DeviceBufferPtr& key = s->relinFor(ell);
            const int tier = key->ksTier;
            const uint32_t n = s->n, K = s->Kof(tier), beta = (ell + s->alpha - 1) / s->alpha;
            const size_t stride = (size_t)(ell + K) * n;
            Ct out = newCt(cc, level + 1, slots);
            auto acc = s->alloc(2 * stride);
            auto ext = s->alloc(stride * beta);
            auto scratch = s->alloc((size_t)2 * ell * n);
            auto& convs = modupConv(cc, ell, tier);
            if (sfp_mult_relin_rescale(s->dev, out->c0, out->c1, a0, a1, b0, b1, ell, K, s->Lq, s->alpha,
                                       convs.data(), key->ptr, s->moddownConvOf(tier), s->pInvModQof(tier),
                                       s->pModQof(tier), s->qInvTable[ell].data(), acc->ptr, ext->ptr,
                                       scratch->ptr) == 0) {
                s->stats.keyswitch++;
                s->stats.rescale++;
                s->countBytes((3.0 * ell + 2.0 * beta * (ell + K)) * n * 8);
                s->countBytes(4.0 * ell * n * 8);
                return out;
            }
        }
        auto t = s->alloc(3 * pw);
        uint64_t* d0 = t->ptr;
        uint64_t* d1 = d0 + pw;
        uint64_t* d2 = d1 + pw;
        sfp_tensor(s->dev, d0, d1, d2, a0, a1, b0, b1, s->qmap(ell));
        return relinRescale(cc, d0, d1, d2, level, slots);
    }

    // multRelinRescale of up to SFP_BATCH_MAX independent operand pairs at one
    // level as ONE batched op (sfp_batch_*): each pair's fused chain is issued
    // on its own virtual lane and the pairs' identical launches run merged.
    // Every pair's buffers live until the batch is issued.  Pairs the backend
    // cannot fuse run one by one (multRelinRescale: the same values).
    static std::vector<Ct> multRelinRescaleMany(CC* cc, const std::vector<const CiphertextImpl<DCRTPoly>*>& a,
                                                const std::vector<const CiphertextImpl<DCRTPoly>*>& b, uint32_t level,
                                                const std::vector<uint32_t>& slots) {
        SfheContextState* s = cc->st.get();
        const size_t cnt = a.size();
        const uint32_t ell = s->ellOf(level);
        std::vector<Ct> out(cnt);
        if (ell < 2) SFHE_THROW("no levels left to rescale (multiplicative depth exhausted)");
        const DeviceBufferPtr& key = s->relinFor(ell);
        const int tier = key->ksTier;
        const uint32_t n = s->n, K = s->Kof(tier), beta = (ell + s->alpha - 1) / s->alpha;
        const size_t stride = (size_t)(ell + K) * n;
        auto& convs = modupConv(cc, ell, tier);
        size_t done = 0;
        {  // (the batch ends here: unfused pairs below run as ordinary ops on the caller's lane)
        BatchScope bs(cc, s->shardAt(ell) ? 0 : (uint32_t)cnt);
        if (bs) {
            for (; done < cnt; ++done) {
                out[done] = newCt(cc, level + 1, slots[done]);
                auto acc = s->alloc(2 * stride);
                auto ext = s->alloc(stride * beta);
                auto scratch = s->alloc((size_t)2 * ell * n);
                bs.lane((uint32_t)done);
                if (sfp_mult_relin_rescale(s->dev, out[done]->c0, out[done]->c1, a[done]->c0, a[done]->c1,
                                           b[done]->c0, b[done]->c1, ell, K, s->Lq, s->alpha, convs.data(),
                                           key->ptr, s->moddownConvOf(tier), s->pInvModQof(tier), s->pModQof(tier),
                                           s->qInvTable[ell].data(), acc->ptr, ext->ptr, scratch->ptr) != 0)
                    break;  // (no fused form: nothing issued for this pair)
                s->stats.keyswitch++;
                s->stats.rescale++;
                s->countBytes((3.0 * ell + 2.0 * beta * (ell + K)) * n * 8);
                s->countBytes(4.0 * ell * n * 8);
            }
        }
        }
        for (size_t i = done; i < cnt; ++i)
            out[i] = multRelinRescale(cc, a[i]->c0, a[i]->c1, b[i]->c0, b[i]->c1, level, slots[i]);
        return out;
    }

    // gal != 0 (hoisted rotations, unsharded levels): ext is the unpermuted
    // ModUp and the inner product reads it through X -> X^gal
    static void innerAndModDown(CC* cc, const uint64_t* ext, size_t stride, uint32_t beta,
                                uint32_t ell, const DeviceBufferPtr& key, uint64_t* out0,
                                uint64_t* out1, int add0, int add1, uint32_t gal = 0) {
        SfheContextState* s = cc->st.get();
        if (s->shardAt(ell)) {
            if (gal) SFHE_THROW("internal: a permuted inner product at a sharded level");
            return innerModDownShard(s, ext, stride, beta, ell, key, out0, out1, add0, add1);
        }
        const int tier = key->ksTier;
        const uint32_t n = s->n, K = s->Kof(tier);
        const size_t accStride = (size_t)(ell + K) * n;
        if (stride != accStride) SFHE_THROW("internal: extended digits of another special-prime tier");
        auto acc = s->alloc(2 * accStride);
        if (gal)
            sfp_ks_inner_aut(s->dev, acc->ptr, acc->ptr + accStride, ext, stride, key->ptr, beta, ell, K, s->Lq, gal);
        else
            sfp_ks_inner(s->dev, acc->ptr, acc->ptr + accStride, ext, stride, key->ptr, beta, ell, K, s->Lq);
        auto scratch = s->alloc((size_t)2 * ell * n);
        sfp_moddown2(s->dev, out0, out1, acc->ptr, accStride, ell, K, s->Lq, s->moddownConvOf(tier),
                     s->pInvModQof(tier), add0, add1, scratch->ptr, 0);
    }

    // ModUp conversion tables of ell limbs: digit j -> the other q rows and
    // the special primes of tier `tier` (-1: all K)
    static std::vector<sfp_conv*>& modupConv(CC* cc, uint32_t ell, int tier = -1) {
        SfheContextState* s = cc->st.get();
        auto& cache = tier < 0 ? s->modupConv : s->tiers[(size_t)tier].modupConv;
        auto it = cache.find(ell);
        if (it != cache.end()) return it->second;
        std::vector<sfp_conv*> v;
        const uint32_t K = s->Kof(tier);
        uint32_t beta = (ell + s->alpha - 1) / s->alpha;
        for (uint32_t j = 0; j < beta; ++j) {
            uint32_t lo = j * s->alpha, hi = std::min(lo + s->alpha, ell);
            std::vector<uint32_t> src, dst, row;
            for (uint32_t i = lo; i < hi; ++i) src.push_back(i);
            for (uint32_t i = 0; i < ell; ++i)
                if (i < lo || i >= hi) dst.push_back(i);
            for (uint32_t k = 0; k < K; ++k) dst.push_back(s->Lq + k);
            // extended layout: q rows at their index, P row k at ell + k
            for (uint32_t p : dst) row.push_back(p < s->Lq ? p : ell + (p - s->Lq));
            v.push_back(makeConv(s, src, dst, row.data()));
        }
        return cache[ell] = v;
    }

    // Special-prime tiers: for each limb bound b of
    // SFHE_KS_TIERS (default "2,4,6,8,10"; "0": none) up to one digit (b <= alpha),
    // the first K' special primes with P' >= Q_b * 2^20 -- the margin the
    // context's P has over its largest digit -- when K' < K.  Unsharded
    // contexts only (a sharded rank keeps one key slice).
    static void buildTiers(SfheContextState* s) {
        const char* v = std::getenv("SFHE_KS_TIERS");
        const std::string spec = v ? v : "2,4,6,8,10";
        std::vector<uint32_t> bounds;
        for (size_t i = 0; i < spec.size();) {
            size_t j = spec.find(',', i);
            if (j == std::string::npos) j = spec.size();
            const long b = std::strtol(spec.substr(i, j - i).c_str(), nullptr, 10);
            if (b > 0) bounds.push_back((uint32_t)b);
            i = j + 1;
        }
        std::sort(bounds.begin(), bounds.end());
        for (uint32_t b : bounds) {
            if (b > s->alpha || b > s->Lq) break;
            double bits = 0;
            for (uint32_t i = 0; i < b; ++i) bits += std::log2((double)s->primes[i]);
            uint32_t K = 0;
            for (double bp = 0; bp < bits + 20.0 && K < s->K; ++K) bp += std::log2((double)s->primes[s->Lq + K]);
            if (K + 1 >= s->K || (!s->tiers.empty() && K <= s->tiers.back().K)) continue;
            KsTier t;
            t.maxEll = b;
            t.K = K;
            t.pModQ.resize(s->Lq);
            t.pInvModQ.resize(s->Lq);
            for (uint32_t i = 0; i < s->Lq; ++i) {
                const u64 qi = s->primes[i];
                u64 pr = 1;
                for (uint32_t k = 0; k < K; ++k) pr = mulmod(pr, s->primes[s->Lq + k] % qi, qi);
                t.pModQ[i] = pr;
                t.pInvModQ[i] = invmod(pr, qi);
            }
            std::vector<uint32_t> src, dst;
            for (uint32_t k = 0; k < K; ++k) src.push_back(s->Lq + k);
            for (uint32_t i = 0; i < s->Lq; ++i) dst.push_back(i);
            t.moddownConv = makeConv(s, src, dst);
            s->tiers.push_back(std::move(t));
        }
    }
    // the tiers' switching keys for the key of s' (after the context's own;
    // a sharded rank keeps its slice, as of every key)
    static void genTierKeys(CC* cc, const uint64_t* sPrime, const uint64_t* sk, uint32_t gal) {
        SfheContextState* s = cc->st.get();
        for (size_t t = 0; t < s->tiers.size(); ++t) {
            auto key = genSwitchKey(cc, sPrime, sk, (int)t);
            if (gal)
                s->tiers[t].rotKeys[gal] = key;
            else
                s->tiers[t].relinKey = key;
        }
    }

    // keep (optional, one flag per source): a PART of the conversion from
    // src -- its constants those of the whole set (y_i = x_i (S/s_i)^-1 mod
    // s_i, multipliers S/s_i mod t) -- over the kept sources only, or, with
    // zeroRest, over every source with the multipliers of the others zeroed.
    // Parts over complementary sources sum (mod t) to the whole conversion.
    static sfp_conv* makeConv(SfheContextState* s, const std::vector<uint32_t>& src,
                              const std::vector<uint32_t>& dst, const uint32_t* dstRow = nullptr,
                              const std::vector<char>* keep = nullptr, bool zeroRest = false) {
        const uint32_t nsAll = (uint32_t)src.size(), nt = (uint32_t)dst.size();
        std::vector<u64> inv, mod;
        std::vector<uint32_t> used;
        for (uint32_t i = 0; i < nsAll; ++i) {
            const bool kept = !keep || (*keep)[i];
            if (!kept && !zeroRest) continue;
            used.push_back(src[i]);
            u64 qi = s->primes[src[i]];
            u64 prod = 1;
            for (uint32_t k = 0; k < nsAll; ++k)
                if (k != i) prod = mulmod(prod, s->primes[src[k]] % qi, qi);
            inv.push_back(invmod(prod, qi));
            for (uint32_t t = 0; t < nt; ++t) {
                u64 pt = s->primes[dst[t]];
                u64 pr = 1;
                for (uint32_t k = 0; k < nsAll; ++k)
                    if (k != i) pr = mulmod(pr, s->primes[src[k]] % pt, pt);
                mod.push_back(kept ? pr : 0);
            }
        }
        const uint32_t ns = (uint32_t)used.size();
        sfp_conv* c = sfp_upload_conv(s->dev, ns, used.data(), nt, dst.data(), dstRow, inv.data(), mod.data());
        if (!c) {
            const char* e = sfp_last_error(s->dev);
            SFHE_THROW(std::string("base-conversion table upload failed: ") + (e ? e : "unknown"));
        }
        return c;
    }

    // switching key from s' (device, Lq+K limbs, eval domain) to s; tier >= 0:
    // that special-prime tier's key (one digit over the Q primes and P')
    static DeviceBufferPtr genSwitchKey(CC* cc, const uint64_t* sPrime, const uint64_t* sk, int tier = -1) {
        SfheContextState* s = cc->st.get();
        if (s->sharded) {  // every rank builds the whole key (same seed, same words) ...
            DeviceBufferPtr whole;
            {
                FullScope fs(s);
                whole = genSwitchKey(cc, sPrime, sk, tier);
            }
            return s->kgeom.rows ? sliceKey(s, whole, tier) : whole;  // ... and keeps its slice
        }
        const uint32_t n = s->n, NP = s->Lq + s->Kof(tier);
        const uint32_t digits = tier < 0 ? s->dnum : 1;
        const u64* pModQ = s->pModQof(tier);
        const sfp_limbs all{NP, NP, 0};
        auto key = s->alloc((size_t)digits * 2 * NP * n);
        key->ksTier = tier;
        auto tmp = s->alloc((size_t)NP * n);
        std::vector<int64_t> e(n);
        for (uint32_t j = 0; j < digits; ++j) {
            uint64_t* b = key->ptr + (size_t)j * 2 * NP * n;
            uint64_t* a = b + (size_t)NP * n;
            sfp_sample_uniform(s->dev, a, all, s->nextSeed());
            sampleCBD(s, e);
            sfp_load_i64(s->dev, tmp->ptr, e.data(), all);
            sfp_ntt(s->dev, tmp->ptr, all, 0);
            // b = e - a s
            sfp_mul(s->dev, b, a, sk, all);
            sfp_sub(s->dev, b, tmp->ptr, b, all);
            // + P * s' on the digit's q-limbs
            uint32_t lo = j * s->alpha, hi = std::min(lo + s->alpha, s->Lq);
            if (lo >= hi) continue;
            std::vector<u64> pk(pModQ + lo, pModQ + hi);
            sfp_mul_const(s->dev, tmp->ptr, sPrime + (size_t)lo * n, pk.data(),
                          Range(lo, hi - lo));
            sfp_add(s->dev, b + (size_t)lo * n, b + (size_t)lo * n, tmp->ptr, Range(lo, hi - lo));
        }
        return key;
    }

    static void sampleCBD(SfheContextState* s, std::vector<int64_t>& e) {
        uint64_t seed = s->nextSeed();
        for (size_t i = 0; i < e.size(); ++i) {
            uint64_t r = sf_splitmix64(seed + i);
            e[i] = (int64_t)__builtin_popcountll(r & 0xFFFFFull) -
                   (int64_t)__builtin_popcountll((r >> 20) & 0xFFFFFull);
        }
    }
    static void sampleTernary(SfheContextState* s, std::vector<int64_t>& v) {
        uint64_t seed = s->nextSeed();
        for (size_t i = 0; i < v.size(); ++i) {
            uint64_t r = sf_splitmix64(seed + i);
            v[i] = (int64_t)(r % 3) - 1;
        }
    }

    // device encoding of a plaintext at `level` with scale Delta_level
    // An encoding produced on another lane that may still be in flight is
    // waited for (device-side) before use.  Inside a capture, an event
    // recorded before it is dropped (BeginCapture drained the device); one
    // recorded inside it is waited for, which makes it a graph edge.
    static const uint64_t* ready(SfheContextState* s, DeviceBuffer* b) {
        if (b->ready && s->capturing && b->readyEpoch != s->captureEpoch) {
            sfp_event_free(s->dev, b->ready);
            b->ready = nullptr;
        }
        if (b->ready && s->capturing) {
            sfp_event_wait(s->dev, b->ready);
        } else if (b->ready) {
            if (sfp_event_done(s->dev, b->ready)) {
                sfp_event_free(s->dev, b->ready);
                b->ready = nullptr;
            } else {
                sfp_event_wait(s->dev, b->ready);
            }
        }
        return b->ptr;
    }

    // Coefficient-domain rows of pt's encoding at `level` for the rows of map
    // m; values whose scaled coefficients need more than 62 bits are encoded
    // at scale / 2^shift and the residues multiplied by 2^shift mod q_i.
    static void encodeRows(SfheContextState* s, const Plaintext& pt, uint32_t level, uint64_t* dst,
                           sfp_limbs m, std::vector<int64_t>* keep = nullptr) {
        // On the device (sfp_encode: the same FFT, bit for bit, no host
        // synchronisation) unless the values could need the encoder's 2^shift
        // range extension, or a trace wants the host coefficients.
        // SFHE_HOST_ENCODE=1 (read per call) encodes on the host.
        double mx = 0.0;
        bool real = true;
        for (const auto& c : pt->values) {
            mx = std::max(mx, std::max(std::fabs(c.real()), std::fabs(c.imag())));
            real = real && c.imag() == 0.0;
        }
        const char* he = std::getenv("SFHE_HOST_ENCODE");
        const bool host = (he && *he == '1') || keep || !(mx * s->scale[level] < 2.0e18) ||
                          (pt->slots & (pt->slots - 1)) || pt->values.size() > pt->slots;
        if (!host) {
            std::vector<double> v;
            v.reserve(pt->values.size() * (real ? 1 : 2));
            for (const auto& c : pt->values) {
                v.push_back(c.real());
                if (!real) v.push_back(c.imag());
            }
            auto scr = s->alloc((size_t)2 * pt->slots);
            sfp_encode(s->dev, dst, v.data(), (uint32_t)pt->values.size(), real ? 1 : 0, pt->slots, s->scale[level],
                       m, scr->ptr);
            s->stats.dev_encodes++;
            return;
        }
        s->stats.host_encodes++;
        std::vector<int64_t> local;
        std::vector<int64_t>& coeffs = keep ? *keep : local;
        const int shift = ckks_encode(pt->values, pt->slots, s->n, s->scale[level], coeffs);
        sfp_load_i64(s->dev, dst, coeffs.data(), m);
        if (shift) {
            std::vector<u64> k(m.count);
            for (uint32_t i = 0; i < m.count; ++i) {
                const u64 q = s->primes[sfp_prime_of(m, i)];
                k[i] = (u64)(((unsigned __int128)1 << shift) % q);
            }
            sfp_mul_const(s->dev, dst, dst, k.data(), m);
        }
    }

    // an encoding made inside an abandoned capture never ran: it is remade
    static bool staleEnc(SfheContextState* s, const DeviceBufferPtr& b) {
        return b->capEpoch && s->abandonedEpochs.count(b->capEpoch);
    }

    // the context-level cache key of (values, slots, level): four independent
    // FNV lanes over the values' words (one serial multiply chain per word
    // was the cold sort's largest host cost after the encoding moved to the
    // device), folded at the end
    static uint64_t encHash(const Plaintext& pt, uint32_t level) {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
        // the doubles' words are read with memcpy (no type-punned loads)
        const char* wv = reinterpret_cast<const char*>(pt->values.data());
        const size_t nw = 2 * pt->values.size();
        auto word = [wv](size_t i) {
            uint64_t x;
            std::memcpy(&x, wv + 8 * i, 8);
            return x;
        };
        uint64_t ln[4] = {h, h ^ 1, h ^ 2, h ^ 3};
        size_t i = 0;
        for (; i + 4 <= nw; i += 4)
            for (int k = 0; k < 4; ++k) ln[k] = (ln[k] ^ word(i + k)) * 1099511628211ull;
        for (; i < nw; ++i) ln[0] = (ln[0] ^ word(i)) * 1099511628211ull;
        for (int k = 0; k < 4; ++k) mix(ln[k]);
        mix(pt->slots);
        mix(level);
        mix(pt->values.size());
        return h;
    }

    // pt's existing encoding at `level` (its own, or an identical plaintext's
    // from the context cache, then adopted), or nullptr; h: the cache key
    // (computed when the cache is on)
    static DeviceBuffer* findEncoding(SfheContextState* s, const Plaintext& pt, uint32_t level, uint64_t& h,
                                      const uint64_t* hashed = nullptr) {
        auto it = pt->encoded.find(level);
        if (it != pt->encoded.end() && staleEnc(s, it->second)) {
            pt->encoded.erase(it);
            it = pt->encoded.end();
        }
        if (it != pt->encoded.end()) return it->second.get();
        h = 0;
        if (!s->ptCacheOn) return nullptr;
        h = hashed ? *hashed : encHash(pt, level);
        auto ci = s->ptCache.find(h);
        if (ci == s->ptCache.end()) return nullptr;
        auto& v = ci->second;
        for (auto e = v.begin(); e != v.end();)
            if (staleEnc(s, e->buf)) {
                s->ptCacheBytes -= e->buf->words * 8;
                e = v.erase(e);
            } else {
                ++e;
            }
        for (auto& e : v)
            if (e.slots == pt->slots && e.values == pt->values) {
                pt->encoded[level] = e.buf;
                return e.buf.get();
            }
        return nullptr;
    }

    // a new encoding of pt at `level` (its evaluation-domain rows in buf)
    static void keepEncoding(SfheContextState* s, const Plaintext& pt, uint32_t level, uint64_t h,
                             const DeviceBufferPtr& buf) {
        buf->ready = sfp_event_record(s->dev);
        buf->readyEpoch = s->capturing ? s->captureEpoch : 0;
        pt->encoded[level] = buf;
        if (s->ptCacheOn && s->ptCacheBytes + buf->words * 8 <= s->ptCacheLimit) {
            s->ptCache[h].push_back(PtCacheEntry{pt->values, pt->slots, buf});
            s->ptCacheBytes += buf->words * 8;
        }
    }

    static const uint64_t* encoded(CC* cc, const Plaintext& pt, uint32_t level) {
        SfheContextState* s = cc->st.get();
        std::lock_guard<std::mutex> g(pt->encMutex);
        uint32_t ell = s->ellOf(level);
        if (s->fullScope && s->rows(ell) != ell) SFHE_THROW("internal: encoding scope");
        if (s->fullScope) {  // every row, uncached (a sharded context caches local rows)
            auto buf = s->alloc(s->polyWords(level));
            encodeRows(s, pt, level, buf->ptr, s->qmap(ell));
            sfp_ntt(s->dev, buf->ptr, s->qmap(ell), 0);
            s->scopeKeep.push_back(buf);
            return buf->ptr;
        }
        uint64_t h = 0;
        if (DeviceBuffer* b = findEncoding(s, pt, level, h)) return ready(s, b);
        std::vector<int64_t> coeffs;
        const size_t pw = s->polyWords(level);
        auto buf = s->alloc(pw);
        static const bool trace = std::getenv("SFHE_TRACE") != nullptr;
        encodeRows(s, pt, level, buf->ptr, s->qmap(ell), trace ? &coeffs : nullptr);
        if (trace) {
            uint64_t f = 1469598103934665603ull;
            for (int64_t v : coeffs) f = (f ^ (uint64_t)v) * 1099511628211ull;
            std::vector<u64> hv(pw);
            sfp_d2h(s->dev, hv.data(), buf->ptr, hv.size() * 8);
            uint64_t gg = 1469598103934665603ull;
            for (u64 v : hv) gg = (gg ^ v) * 1099511628211ull;
            std::fprintf(stderr, "ENCODE slots=%u level=%u coeffs=%016llx loaded=%016llx\n", pt->slots,
                         level, (unsigned long long)f, (unsigned long long)gg);
        }
        sfp_ntt(s->dev, buf->ptr, s->qmap(ell), 0);
        keepEncoding(s, pt, level, h, buf);
        return buf->ptr;
    }

    // Every not-yet-encoded plaintext of `pts` at `level` (one slot count,
    // value count and real-ness: the sort's masks of one giant step) encoded
    // in ONE batch -- one launch per encoder stage and one NTT launch pair
    // for all of them -- into views of one pool block.  The same values as
    // encoded() one at a time (sfp_encode_batch is sfp_encode per batch
    // member); the cold sort's mask encodings were ~10 launches each.
    static void encodeBatch(CC* cc, const std::vector<Plaintext>& pts, uint32_t level) {
        SfheContextState* s = cc->st.get();
        if (pts.size() < 2 || s->fullScope) return;
        static const bool trace = std::getenv("SFHE_TRACE") != nullptr;
        const char* he = std::getenv("SFHE_HOST_ENCODE");
        if (trace || (he && *he == '1')) return;
        const uint32_t ell = s->ellOf(level);
        const size_t pw = s->polyWords(level);
        struct Miss {
            Plaintext pt;
            uint64_t h;
        };
        std::vector<Miss> miss;
        bool real0 = true;
        // the cache keys and value ranges of every plaintext over the host's
        // cores (each a pass over 2 * slots words)
        std::vector<uint64_t> hs(pts.size(), 0);
        std::vector<double> mxs(pts.size(), 0.0);
        std::vector<char> reals(pts.size(), 1), scanned(pts.size(), 0);
        auto scan = [&](size_t i) {
            if (s->ptCacheOn) hs[i] = encHash(pts[i], level);
            double mx = 0.0;
            bool real = true;
            for (const auto& c : pts[i]->values) {
                mx = std::max(mx, std::max(std::fabs(c.real()), std::fabs(c.imag())));
                real = real && c.imag() == 0.0;
            }
            mxs[i] = mx;
            reals[i] = real;
            scanned[i] = 1;
        };
        ParallelFor(
            pts.size(),
            [&](size_t i) {
                if (pts[i] && !pts[i]->encoded.count(level)) scan(i);  // (encoded ones: no pass at all)
            },
            2);
        for (size_t pi = 0; pi < pts.size(); ++pi) {
            const auto& pt = pts[pi];
            if (!pt) continue;
            std::lock_guard<std::mutex> g(pt->encMutex);
            uint64_t h = 0;
            if (findEncoding(s, pt, level, h, scanned[pi] && s->ptCacheOn ? &hs[pi] : nullptr)) continue;
            if (!scanned[pi]) scan(pi);  // its own encoding was stale (an abandoned capture's)
            bool dup = false;  // the same plaintext twice in the list
            for (auto& m : miss) dup = dup || m.pt == pt;
            if (dup) continue;
            const double mx = mxs[pi];
            const bool real = reals[pi] != 0;
            // the device path of encodeRows, and the shape of the first miss
            if (!(mx * s->scale[level] < 2.0e18) || (pt->slots & (pt->slots - 1)) ||
                pt->values.size() > pt->slots)
                continue;
            if (!miss.empty() && (pt->slots != miss[0].pt->slots ||
                                  pt->values.size() != miss[0].pt->values.size() || real != real0))
                continue;
            if (miss.empty()) real0 = real;
            miss.push_back({pt, h});
        }
        if (miss.size() < 2) return;
        const uint32_t count = (uint32_t)miss.size(), slots = miss[0].pt->slots;
        const uint32_t nvals = (uint32_t)miss[0].pt->values.size();
        std::vector<double> vals;
        vals.reserve((size_t)count * nvals * (real0 ? 1 : 2));
        for (auto& m : miss)
            for (const auto& c : m.pt->values) {
                vals.push_back(c.real());
                if (!real0) vals.push_back(c.imag());
            }
        auto block = s->alloc((size_t)count * pw);
        auto scr = s->alloc((size_t)count * 2 * slots);
        sfp_encode_batch(s->dev, block->ptr, pw, vals.data(), nvals, count, real0 ? 1 : 0, slots, s->scale[level],
                         s->qmap(ell), scr->ptr);
        sfp_ntt_batch(s->dev, block->ptr, pw, count, s->qmap(ell), 0);
        s->stats.dev_encodes += count;
        for (uint32_t b = 0; b < count; ++b) {
            auto view = std::make_shared<DeviceBuffer>(s, block->ptr + (size_t)b * pw, pw, block->lane, block->region);
            view->parent = block;
            view->seq = block->seq;
            view->capEpoch = block->capEpoch;
            std::lock_guard<std::mutex> g(miss[b].pt->encMutex);
            keepEncoding(s, miss[b].pt, level, miss[b].h, view);
        }
    }

    // pt at `level` over the extended basis: its ell q rows then the K P rows
    // (evaluation domain), cached on the plaintext beside its q-row encodings
    static const uint64_t* encodedExt(CC* cc, const Plaintext& pt, uint32_t level) {
        SfheContextState* s = cc->st.get();
        if (s->shardAt(s->ellOf(level))) SFHE_THROW("internal: extended-basis encodings are unsharded");
        std::lock_guard<std::mutex> g(pt->encMutex);
        const uint32_t key = level | 0x40000000u;
        auto stale = [&](const DeviceBufferPtr& b) { return b->capEpoch && s->abandonedEpochs.count(b->capEpoch); };
        auto it = pt->encoded.find(key);
        if (it != pt->encoded.end() && stale(it->second)) {
            pt->encoded.erase(it);
            it = pt->encoded.end();
        }
        if (it != pt->encoded.end()) return ready(s, it->second.get());
        const uint32_t ell = s->ellOf(level);
        const sfp_limbs m{ell + s->K, ell, s->Lq};
        auto buf = s->alloc((size_t)m.count * s->n);
        encodeRows(s, pt, level, buf->ptr, m);
        sfp_ntt(s->dev, buf->ptr, m, 0);
        buf->ready = sfp_event_record(s->dev);
        buf->readyEpoch = s->capturing ? s->captureEpoch : 0;
        pt->encoded[key] = buf;
        return buf->ptr;
    }

    // a canonical ciphertext over existing rows (deferred ops keep the rows
    // they were given pinned, never the caller's possibly reassigned handle)
    static Ct view(CC* cc, const DeviceBufferPtr& buf, uint64_t* c0, uint64_t* c1, uint32_t level, double scale,
                   uint32_t slots) {
        auto ct = std::make_shared<CiphertextImpl<DCRTPoly>>();
        ct->cc = cc->shared_from_this();
        ct->buf = buf;
        ct->c0 = c0;
        ct->c1 = c1;
        ct->level = level;
        ct->scale = scale;
        ct->slots = slots;
        return ct;
    }
    // fill `dst` (a deferred ciphertext) with the rows of `src`
    static void adopt(CiphertextImpl<DCRTPoly>& dst, const Ct& src) {
        dst.buf = src->buf;
        dst.c0 = src->c0;
        dst.c1 = src->c1;
        dst.scale = src->scale;
        dst.pend = src->pend;
    }
    static void adoptPending(CiphertextImpl<DCRTPoly>& dst, const DeviceBufferPtr& buf, uint64_t* c0,
                             uint64_t* c1) {
        SfheContextState* s = dst.cc->st.get();
        dst.buf = buf;
        dst.c0 = c0;
        dst.c1 = c1;
        dst.pend = true;
        dst.scale = s->preScale(dst.level);
        s->wrote(buf.get());
    }

    static Ct copyOf(CC* cc, const Ct& a) {
        SfheContextState* s = cc->st.get();
        Ct out = a->pend ? newPendingCt(cc, a->level, a->slots) : newCt(cc, a->level, a->slots);
        const size_t pw = s->polyWords(a->pend ? a->level - 1 : a->level);
        size_t bytes = pw * 8;
        if (a->c1 == a->c0 + pw) {  // [c0][c1] packed: one copy
            sfp_d2d(s->dev, out->c0, a->c0, 2 * bytes);
        } else {
            sfp_d2d(s->dev, out->c0, a->c0, bytes);
            sfp_d2d(s->dev, out->c1, a->c1, bytes);
        }
        return out;
    }
    // make `a` exclusively owned before an in-place update
    static void own(CC* cc, Ct& a) {
        if (a->buf.use_count() > 1) {
            Ct c = copyOf(cc, a);
            a->buf = c->buf;
            a->c0 = c->c0;
            a->c1 = c->c1;
        }
    }
};

// ============================================================================
// deferred products (lazy rescaling; see SfheInternal::materialize)

namespace {
using CtI = CiphertextImpl<DCRTPoly>;
using CCI = CryptoContextImpl<DCRTPoly>;

// EvalMult(ct, double): rows x per-row residues K (the constant times the
// product scale), then the rescale
struct DeferredConstMult : DeferredOp {
    DeviceBufferPtr pin;
    uint64_t *c0, *c1;
    uint32_t level, slots;
    double scale;
    std::vector<uint64_t> k;
    void run(CCI* cc, CtI& ct, bool pending) override {
        SfheContextState* s = cc->state();
        s->dep(pin.get());
        if (!pending) {
            auto src = SfheInternal::view(cc, pin, c0, c1, level, scale, slots);
            SfheInternal::adopt(ct, SfheInternal::mulRescale(cc, src, level, k.data(), nullptr, slots));
            return;
        }
        const size_t pw = s->polyWords(level);
        auto out = s->alloc(2 * pw);
        if ((size_t)(c1 - c0) == pw) {  // both polynomials in one launch
            std::vector<uint64_t> kk(k);
            kk.insert(kk.end(), k.begin(), k.end());
            sfp_mul_const(s->dev, out->ptr, c0, kk.data(), SfheInternal::both(s, s->ellOf(level)));
        } else {
            sfp_mul_const(s->dev, out->ptr, c0, k.data(), s->qmap(s->ellOf(level)));
            sfp_mul_const(s->dev, out->ptr + pw, c1, k.data(), s->qmap(s->ellOf(level)));
        }
        SfheInternal::adoptPending(ct, out, out->ptr, out->ptr + pw);
    }
};

// EvalMult(ct, pt): rows (.) the plaintext's encoding at `level`
struct DeferredPlainMult : DeferredOp {
    DeviceBufferPtr pin;
    uint64_t *c0, *c1;
    uint32_t level, slots;
    double scale;
    Plaintext pt;
    void run(CCI* cc, CtI& ct, bool pending) override {
        SfheContextState* s = cc->state();
        s->dep(pin.get());
        const uint64_t* m = SfheInternal::encoded(cc, pt, level);
        if (!pending) {
            auto src = SfheInternal::view(cc, pin, c0, c1, level, scale, slots);
            SfheInternal::adopt(ct, SfheInternal::mulRescale(cc, src, level, nullptr, m, slots));
            return;
        }
        const size_t pw = s->polyWords(level);
        auto out = s->alloc(2 * pw);
        sfp_mul(s->dev, out->ptr, c0, m, s->qmap(s->ellOf(level)));
        sfp_mul(s->dev, out->ptr + pw, c1, m, s->qmap(s->ellOf(level)));
        SfheInternal::adoptPending(ct, out, out->ptr, out->ptr + pw);
    }
};

// EvalMultAddPlain: sum_i a_i (.) p_i, then one rescale
struct DeferredMacPlain : DeferredOp {
    std::vector<DeviceBufferPtr> pins;
    std::vector<const uint64_t*> x0, x1;
    std::vector<Plaintext> pts;
    uint32_t level, slots;
    void run(CCI* cc, CtI& ct, bool pending) override {
        SfheContextState* s = cc->state();
        for (auto& b : pins) s->dep(b.get());
        std::vector<const uint64_t*> m;
        SfheInternal::encodeBatch(cc, pts, level);
        for (auto& p : pts) m.push_back(SfheInternal::encoded(cc, p, level));
        const uint32_t ell = s->ellOf(level);
        const size_t pw = s->polyWords(level);
        auto tmp = s->alloc(2 * pw);
        uint64_t* t0 = tmp->ptr;
        uint64_t* t1 = t0 + pw;
        for (size_t done = 0; done < x0.size(); done += SFP_MAX_WSUM) {
            const uint32_t take = (uint32_t)std::min<size_t>(SFP_MAX_WSUM, x0.size() - done);
            if (done == 0) {
                sfp_mac_plain2(s->dev, t0, t1, x0.data(), x1.data(), m.data(), take, s->qmap(ell));
            } else {
                auto part = s->alloc(2 * pw);
                sfp_mac_plain2(s->dev, part->ptr, part->ptr + pw, x0.data() + done, x1.data() + done,
                               m.data() + done, take, s->qmap(ell));
                sfp_add(s->dev, t0, t0, part->ptr, s->qmap(ell));
                sfp_add(s->dev, t1, t1, part->ptr + pw, s->qmap(ell));
            }
        }
        if (pending) {
            SfheInternal::adoptPending(ct, tmp, t0, t1);
            return;
        }
        SfheInternal::adopt(ct, SfheInternal::rescale(cc, t0, t1, level, slots));
    }
};

// Pending mask sums over the SAME ciphertexts -- the giant steps of one
// baby-step set (vecRotsOpt), the blind rotations' masks over one set of
// masked inputs -- consumed together by EvalRotateSum run as multi-output
// launches of up to SFP_MAC_MULTI_G sums (sfp_mac_plain2_multi): each
// ciphertext row is read once per group instead of once per sum.  The same
// residues as each sum's own DeferredMacPlain::run.  SFHE_MAC_MULTI=0: off.
static void macGroups(CryptoContextImpl<DCRTPoly>* cc, const std::vector<Ciphertext<DCRTPoly>>& a,
                      const std::vector<size_t>& idx) {
    static const bool on = [] {
        const char* v = std::getenv("SFHE_MAC_MULTI");
        return !v || *v != '0';
    }();
    static const size_t maxG = [] {  // SFHE_MAC_MULTI_G: sums per launch (A/B; at most SFP_MAC_MULTI_G)
        const char* v = std::getenv("SFHE_MAC_MULTI_G");
        const int g = v ? std::atoi(v) : SFP_MAC_MULTI_G;
        return (size_t)std::max(2, std::min(g, SFP_MAC_MULTI_G));
    }();
    if (!on) return;
    SfheContextState* s = cc->state();
    auto macOf = [&](size_t k) -> DeferredMacPlain* {
        const auto& c = *a[k];
        if (!c.def || c.undo) return nullptr;
        auto* m = dynamic_cast<DeferredMacPlain*>(c.def.get());
        return (m && !m->x0.empty() && m->x0.size() <= SFP_MAC_MULTI_N) ? m : nullptr;
    };
    std::vector<bool> used(idx.size(), false);
    for (size_t u = 0; u < idx.size(); ++u) {
        DeferredMacPlain* m0 = used[u] ? nullptr : macOf(idx[u]);
        if (!m0) continue;
        std::vector<size_t> grp{u};
        for (size_t v = u + 1; v < idx.size() && grp.size() < maxG; ++v) {
            DeferredMacPlain* m = used[v] ? nullptr : macOf(idx[v]);
            if (m && m->level == m0->level && m->x0 == m0->x0 && m->x1 == m0->x1) grp.push_back(v);
        }
        if (grp.size() < 2) continue;
        const uint32_t level = m0->level, nin = (uint32_t)m0->x0.size(), ng = (uint32_t)grp.size();
        std::vector<std::shared_ptr<DeferredOp>> defs;  // (each keeps its pins alive until the launch)
        std::vector<Plaintext> pts;
        for (size_t g : grp) {
            used[g] = true;
            defs.push_back(SfheInternal::takeDeferred(*a[idx[g]], true));
            auto* m = static_cast<DeferredMacPlain*>(defs.back().get());
            for (auto& b : m->pins) s->dep(b.get());
            pts.insert(pts.end(), m->pts.begin(), m->pts.end());
        }
        SfheInternal::encodeBatch(cc, pts, level);
        std::vector<const uint64_t*> mm;
        for (auto& p : pts) mm.push_back(SfheInternal::encoded(cc, p, level));
        const uint32_t ell = s->ellOf(level);
        const size_t pw = s->polyWords(level);
        std::vector<DeviceBufferPtr> bufs;
        std::vector<uint64_t*> o0, o1;
        for (uint32_t g = 0; g < ng; ++g) {
            bufs.push_back(s->alloc(2 * pw));
            o0.push_back(bufs.back()->ptr);
            o1.push_back(bufs.back()->ptr + pw);
        }
        const auto* x = static_cast<DeferredMacPlain*>(defs[0].get());
        if (sfp_mac_plain2_multi(s->dev, o0.data(), o1.data(), x->x0.data(), x->x1.data(), mm.data(), nin, ng,
                                 s->qmap(ell)) != 0)
            for (uint32_t g = 0; g < ng; ++g)
                sfp_mac_plain2(s->dev, o0[g], o1[g], x->x0.data(), x->x1.data(), mm.data() + (size_t)g * nin, nin,
                               s->qmap(ell));
        for (uint32_t g = 0; g < ng; ++g) SfheInternal::adoptPending(*a[idx[grp[g]]], bufs[g], o0[g], o1[g]);
    }
}

// EvalMult(ct, ct): the tensor, relinearisation and rescale deferred to the
// first consumer (the canonical form runs them as one fused chain,
// multRelinRescale; the pending form needs the tensor's rows)
struct DeferredRelin : DeferredOp {
    DeviceBufferPtr pa, pb;  // the aligned operands' rows, pinned
    const uint64_t *a0, *a1, *b0, *b1;
    uint32_t level, slots;
    void run(CCI* cc, CtI& ct, bool pending) override {
        SfheContextState* s = cc->state();
        s->dep(pa.get());
        s->dep(pb.get());
        if (!pending) {
            SfheInternal::adopt(ct, SfheInternal::multRelinRescale(cc, a0, a1, b0, b1, level, slots));
            return;
        }
        const size_t pw = s->polyWords(level);
        auto t = s->alloc(3 * pw);
        uint64_t* d0 = t->ptr;
        uint64_t* d1 = d0 + pw;
        uint64_t* d2 = d1 + pw;
        sfp_tensor(s->dev, d0, d1, d2, a0, a1, b0, b1, s->qmap(s->ellOf(level)));
        SfheInternal::keySwitch(cc, d2, s->ellOf(level), s->relinFor(s->ellOf(level)), d0, d1, 1, 1);
        SfheInternal::adoptPending(ct, t, d0, d1);
    }
};
}  // namespace

// ============================================================================
// context construction

// contexts alive in this process (diagnostics: sfhe_live_contexts)
static std::atomic<int> g_liveContexts{0};
int CryptoContextImpl<DCRTPoly>::LiveContexts() { return g_liveContexts.load(); }

void SfheCheckLayout(uint64_t callerStamp) {
    const uint64_t mine = SfheFacadeLayout();
    if (callerStamp == mine) return;
    char b[160];
    std::snprintf(b, sizeof b, "caller stamp %016llx, library stamp %016llx (facade ABI version %d)",
                  (unsigned long long)callerStamp, (unsigned long long)mine, SFHE_FACADE_ABI_VERSION);
    SFHE_THROW(std::string("the engine headers this program was compiled against do not match the library's "
                           "(object layouts differ; rebuild the program against the installed headers): ") + b);
}

CryptoContextImpl<DCRTPoly>::CryptoContextImpl(const CCParams<CryptoContextCKKSRNS>& p)
    : st(new SfheContextState) {
    SfheContextState& s = *st;
    s.params = p;
    s.L = p.GetMultiplicativeDepth();
    s.Lq = s.L + 1;
    s.seed = p.GetSeed();
    switch (p.GetScalingTechnique()) {
        case FLEXIBLEAUTO: s.ext = false; break;
        case FLEXIBLEAUTOEXT: s.ext = true; break;
        default: SFHE_THROW("only FLEXIBLEAUTO and FLEXIBLEAUTOEXT scaling are supported");
    }
    const uint32_t sbits = p.GetScalingModSize();
    const uint32_t fbits = p.GetFirstModSize();
    if (sbits < 20 || sbits > 60) SFHE_THROW("scaling mod size must be in [20, 60]");
    if (fbits < sbits || fbits > 60) SFHE_THROW("first mod size must be in [scale bits, 60]");
    s.dnum = p.GetNumLargeDigits();
    if (s.dnum == 0 && std::getenv("SFHE_DNUM")) s.dnum = (uint32_t)std::atoi(std::getenv("SFHE_DNUM"));  // (A/B)
    if (s.dnum == 0) s.dnum = s.Lq > 3 ? 3 : std::max<uint32_t>(1, s.Lq);
    s.dnum = std::min(s.dnum, s.Lq);
    s.alpha = (s.Lq + s.dnum - 1) / s.dnum;
    s.dnum = (s.Lq + s.alpha - 1) / s.alpha;

    uint32_t n = p.GetRingDim();
    uint32_t batch = p.GetBatchSize();
    bool secure = p.GetSecurityLevel() != HEStd_NotSet;
    uint32_t logn_lo = 10;
    if (n) {
        if (n & (n - 1)) SFHE_THROW("ring dimension must be a power of two");
        logn_lo = (uint32_t)__builtin_ctz(n);
    } else if (batch) {
        while ((1u << logn_lo) < 2 * batch) ++logn_lo;
    }
    for (uint32_t logn = logn_lo;; ++logn) {
        if (logn > 17 && !n) SFHE_THROW("no ring dimension <= 2^17 satisfies the parameters");
        const uint32_t N = 1u << logn;
        const u64 m = 2ull * N;
        std::set<u64> used;
        std::vector<u64> q(s.Lq);
        q[0] = primeBelow(1ull << fbits, m, used);
        used.insert(q[0]);
        std::vector<double> sc(s.Lq);
        sc[0] = std::ldexp(1.0, (int)sbits);
        for (uint32_t l = 0; l < s.L; ++l) {
            double target = sc[l] * sc[l] / std::ldexp(1.0, (int)sbits);
            u64 pr = primeNear(target, m, used);
            used.insert(pr);
            q[s.L - l] = pr;
            sc[l + 1] = sc[l] * sc[l] / (double)pr;
        }
        // special primes: enough bits to cover the largest digit
        double maxDigitBits = 0;
        for (uint32_t j = 0; j < s.dnum; ++j) {
            double b = 0;
            for (uint32_t i = j * s.alpha; i < std::min((j + 1) * s.alpha, s.Lq); ++i)
                b += std::log2((double)q[i]);
            maxDigitBits = std::max(maxDigitBits, b);
        }
        // P must exceed every digit modulus with margin, or the key-switch
        // noise (digit * error / P) is not negligible.  The special primes
        // sit just below 2^42 when the scaling primes do (so every row but
        // q_0 takes the device's FP64 arithmetic: NTT, base conversion),
        // just below 2^60 otherwise.
        const u64 pTop = sbits <= 41 ? (1ull << 42) : (1ull << 60);
        std::vector<u64> P;
        u64 bound = pTop;
        for (double bitsP = 0; bitsP < maxDigitBits + 20.0;) {
            u64 pr = primeBelow(bound, m, used);
            used.insert(pr);
            P.push_back(pr);
            bitsP += std::log2((double)pr);
            bound = pr;
        }
        const uint32_t K = (uint32_t)P.size();
        u64 qext = 0;
        if (s.ext) {
            qext = primeNear(std::ldexp(1.0, (int)sbits), m, used);
            used.insert(qext);
        }
        double logQP = qext ? std::log2((double)qext) : 0.0;
        for (u64 x : q) logQP += std::log2((double)x);
        for (u64 x : P) logQP += std::log2((double)x);
        if (secure && logQP > maxLogQ128(logn)) {
            if (n)
                SFHE_THROW("The specified ring dimension (" + std::to_string(n) +
                           ") does not comply with the HE standard recommendation (log2 QP = " +
                           std::to_string(logQP) + " > " + std::to_string(maxLogQ128(logn)) +
                           "); use HEStd_NotSet or a larger ring");
            continue;
        }
        s.n = N;
        s.logn = logn;
        s.K = K;
        s.primes = q;
        s.primes.insert(s.primes.end(), P.begin(), P.end());
        if (s.ext) s.primes.push_back(qext);
        s.scale = sc;
        break;
    }
    s.batch = batch ? batch : s.n / 2;
    if (std::getenv("SFHE_NO_PTCACHE")) s.ptCacheOn = false;
    if (s.batch > s.n / 2) SFHE_THROW("batch size exceeds n/2");

    const uint32_t NP = s.tablePrimes();
    for (u64 x : s.primes) s.bar.push_back(sf_make_barrett(x));

    // NTT tables
    std::vector<u64> psi((size_t)NP * s.n), psiS((size_t)NP * s.n), ipsi((size_t)NP * s.n),
        ipsiS((size_t)NP * s.n), ninv(NP), ninvS(NP);
    for (uint32_t i = 0; i < NP; ++i) {
        u64 q = s.primes[i];
        u64 w = findPsi(q, s.n);
        u64 wi = invmod(w, q);
        std::vector<u64> pw(s.n), ipw(s.n);
        pw[0] = ipw[0] = 1;
        for (uint32_t k = 1; k < s.n; ++k) {
            pw[k] = mulmod(pw[k - 1], w, q);
            ipw[k] = mulmod(ipw[k - 1], wi, q);
        }
        for (uint32_t k = 0; k < s.n; ++k) {
            uint32_t r = sf_brev(k, s.logn);
            size_t o = (size_t)i * s.n + k;
            psi[o] = pw[r];
            psiS[o] = sf_shoup_precomp(pw[r], q);
            ipsi[o] = ipw[r];
            ipsiS[o] = sf_shoup_precomp(ipw[r], q);
        }
        ninv[i] = invmod(s.n % q, q);
        ninvS[i] = sf_shoup_precomp(ninv[i], q);
    }
    sfp_tables t;
    t.logn = s.logn;
    t.nprimes = NP;
    t.primes = s.primes.data();
    t.psi_rev = psi.data();
    t.psi_rev_shoup = psiS.data();
    t.ipsi_rev = ipsi.data();
    t.ipsi_rev_shoup = ipsiS.data();
    t.n_inv = ninv.data();
    t.n_inv_shoup = ninvS.data();
    s.dev = sfp_create(p.GetDevice(), &t);
    if (!s.dev) SFHE_THROW(std::string("device backend '") + sfp_backend_name() + "' failed to initialise");
    {  // the device encoder works from the host encoder's own tables
        const uint64_t* rot = nullptr;
        const double* ksi = nullptr;
        ckks_encoder_tables(s.n, &rot, &ksi);
        sfp_encode_setup(s.dev, rot, ksi);
    }

    if (s.ext) {
        s.extIdx = s.Lq + s.K;
        const u64 qe = s.primes[s.extIdx];
        for (uint32_t i = 0; i < s.Lq; ++i) {
            s.extModQ.push_back(qe % s.primes[i]);
            s.extInvModQ.push_back(invmod(qe % s.primes[i], s.primes[i]));
        }
    }
    // P mod q_i, P^{-1} mod q_i
    s.pModQ.resize(s.Lq);
    s.pInvModQ.resize(s.Lq);
    for (uint32_t i = 0; i < s.Lq; ++i) {
        u64 qi = s.primes[i], pr = 1;
        for (uint32_t k = 0; k < s.K; ++k) pr = mulmod(pr, s.primes[s.Lq + k] % qi, qi);
        s.pModQ[i] = pr;
        s.pInvModQ[i] = invmod(pr, qi);
    }
    {
        std::vector<uint32_t> src, dst;
        for (uint32_t k = 0; k < s.K; ++k) src.push_back(s.Lq + k);
        for (uint32_t i = 0; i < s.Lq; ++i) dst.push_back(i);
        s.moddownConv = SfheInternal::makeConv(&s, src, dst);
    }
    SfheInternal::buildTiers(&s);
    s.qInvTable.resize(s.Lq + 1);
    for (uint32_t ell = 2; ell <= s.Lq; ++ell) {
        u64 ql = s.primes[ell - 1];
        for (uint32_t i = 0; i + 1 < ell; ++i)
            s.qInvTable[ell].push_back(invmod(ql % s.primes[i], s.primes[i]));
    }
    g_liveContexts.fetch_add(1);
}

CryptoContextImpl<DCRTPoly>::~CryptoContextImpl() {
    if (!st) return;
    g_liveContexts.fetch_sub(1);
    st->relinKey.reset();
    st->rotKeys.clear();
    for (auto& t : st->tiers) {
        t.relinKey.reset();
        t.rotKeys.clear();
        for (auto& kv : t.modupConv)
            for (auto* c : kv.second) sfp_free_conv(st->dev, c);
        if (t.moddownConv) sfp_free_conv(st->dev, t.moddownConv);
    }
    st->ptCache.clear();
    releaseBootstrapGraphs();  // the replay graphs' blocks back to the pool first
    st->boot.clear();  // its diagonal encodings return blocks to the pool below
    for (auto& kv : st->modupConv)
        for (auto* c : kv.second) sfp_free_conv(st->dev, c);
    if (st->moddownConv) sfp_free_conv(st->dev, st->moddownConv);
    for (auto& kv : st->modupConvShard)
        for (auto* c : kv.second) sfp_free_conv(st->dev, c);
    for (auto& kv : st->modupConvSplit)
        for (auto& pr : kv.second) {
            sfp_free_conv(st->dev, pr.first);
            sfp_free_conv(st->dev, pr.second);
        }
    if (st->moddownConvShard) sfp_free_conv(st->dev, st->moddownConvShard);
    st->releaseAll();
    sfp_destroy(st->dev);
}

uint32_t CryptoContextImpl<DCRTPoly>::GetRingDimension() const { return st->n; }
uint32_t CryptoContextImpl<DCRTPoly>::GetMultiplicativeDepth() const { return st->L; }
EncodingParams CryptoContextImpl<DCRTPoly>::GetEncodingParams() const {
    return std::make_shared<EncodingParamsImpl>(st->batch);
}

uint32_t CryptoContextImpl<DCRTPoly>::GaloisForRotation(int32_t r) const {
    const int64_t half = st->n / 2;
    int64_t rr = ((int64_t)r % half + half) % half;
    return (uint32_t)powmod(5, (u64)rr, 2ull * st->n);
}

bool CryptoContextImpl<DCRTPoly>::HasRotationKey(int32_t r) const {
    return st->rotKeys.count(GaloisForRotation(r)) > 0;
}

void CryptoContextImpl<DCRTPoly>::Synchronize() {
    sfp_sync(st->dev);
    const char* e = sfp_last_error(st->dev);
    if (e) SFHE_THROW(std::string("device error: ") + e);
}

// a sharded context issues its collectives in program order on one lane
int CryptoContextImpl<DCRTPoly>::LaneCount() const { return st->sharded ? 1 : sfp_lanes(st->dev); }

void CryptoContextImpl<DCRTPoly>::ForkLanes(int count, bool stacked) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (s->forkedLanes) SFHE_THROW("ForkLanes: a lane region is already open");
    count = std::max(1, std::min(count, sfp_lanes(s->dev)));
    sfp_set_lane(s->dev, 0);
    s->lane = 0;
    s->setMyLane(0);
    for (int i = 1; i < count; ++i) s->laneWait(i, 0);
    {
        std::lock_guard<std::mutex> pg(s->poolMu);
        for (auto& kv : s->freeList[0])
            for (auto* p : kv.second) s->forkPool[kv.first].push_back(p);
        s->freeList[0].clear();
    }
    s->forkedLanes = count;
    s->region = ++s->regionCount;
    if (stacked && count > 1) sfp_stack_begin(s->dev);
}

void CryptoContextImpl<DCRTPoly>::SetLane(int lane) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (lane != 0 && (!s->forkedLanes || lane >= s->forkedLanes))
        SFHE_THROW("SetLane: lane " + std::to_string(lane) + " outside the open region");
    if (lane < 0 || lane >= sfp_lanes(s->dev)) SFHE_THROW("SetLane: no lane " + std::to_string(lane));
    s->setMyLane(lane);
    s->lane = lane;
    sfp_set_lane(s->dev, lane);
}

void CryptoContextImpl<DCRTPoly>::JoinLanes() {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (!s->forkedLanes) return;
    static const bool stats = std::getenv("SFHE_LANE_STATS") != nullptr;
    if (stats) {
        std::fprintf(stderr, "LANESTATS region %llu: %llu data-dependency waits across lanes\n", (unsigned long long)s->region,
                     (unsigned long long)s->regionDepWaits);
        s->regionDepWaits = 0;
    }
    sfp_stack_end(s->dev);  // (a stacked region: its launches are issued now, on lane 0)
    for (int i = 1; i < s->forkedLanes; ++i) s->laneWait(0, i);
    sfp_set_lane(s->dev, 0);
    std::lock_guard<std::mutex> pg(s->poolMu);
    for (int i = 1; i < s->forkedLanes; ++i) {
        for (auto& kv : s->freeList[i])
            for (auto* p : kv.second) s->freeList[0][kv.first].push_back(p);
        s->freeList[i].clear();
    }
    for (auto& e : s->deferredFree) s->freeList[0][e.first].push_back(e.second);
    s->deferredFree.clear();
    for (auto& kv : s->forkPool)
        for (auto* p : kv.second) s->freeList[0][kv.first].push_back(p);
    s->forkPool.clear();
    s->lane = 0;
    s->setMyLane(0);
    s->forkedLanes = 0;
    s->region = 0;
}

bool CryptoContextImpl<DCRTPoly>::BeginBatch(uint32_t count) {
    SfheContextState* s = st.get();
    s->opMu.lock();  // held until EndBatch: no other host thread issues in between
    {
        OpLock g(s);
        if (!s->batchDepth && sfp_batch_begin(s->dev, count)) {
            std::lock_guard<std::mutex> pg(s->poolMu);
            ++s->batchDepth;
            s->batchThread = std::this_thread::get_id();
            return true;
        }
    }
    s->opMu.unlock();
    return false;
}

uint32_t CryptoContextImpl<DCRTPoly>::BatchWidth() const { return batchWidth(); }

void CryptoContextImpl<DCRTPoly>::BatchLane(uint32_t i) {
    OpLock g(st.get());
    if (st->batchDepth) sfp_batch_lane(st->dev, i);
}

void CryptoContextImpl<DCRTPoly>::EndBatch() {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (!s->batchDepth) return;
    sfp_batch_end(s->dev);  // every op of the batch is issued on this lane now
    std::lock_guard<std::mutex> pg(s->poolMu);
    --s->batchDepth;
    // (this thread freed them: the same lane test ~DeviceBuffer applies)
    for (auto& e : s->batchFree) s->poolReturn(e.words, e.ptr, e.lane, e.region, s->myLane());
    s->batchFree.clear();
    s->opMu.unlock();  // (BeginBatch's)
}

void CryptoContextImpl<DCRTPoly>::SetPlaintextCache(bool on) {
    OpLock g(st.get());
    st->ptCacheOn = on;
    if (!on) {
        st->ptCache.clear();
        st->ptCacheBytes = 0;
    }
}

CryptoContextImpl<DCRTPoly>::OpStats CryptoContextImpl<DCRTPoly>::GetOpStats() const {
    OpStats o = st->stats;
    std::lock_guard<std::mutex> g(st->poolMu);
    o.pool_bytes = st->poolBytes;
    return o;
}
void CryptoContextImpl<DCRTPoly>::ResetOpStats() { st->stats = OpStats(); }

// ============================================================================
// keys

std::string KeyTagString(uint64_t tag) {
    char b[17];
    std::snprintf(b, sizeof b, "%016llx", (unsigned long long)tag);
    return b;
}

uint64_t CryptoContextImpl<DCRTPoly>::KeyTag() const { return st->keyTag; }

KeyPair<DCRTPoly> CryptoContextImpl<DCRTPoly>::KeyGen() {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    FullScope fs(s);  // secret and public keys keep every row (sharding: setup only)
    const uint32_t NP = s->Lq + s->K;
    KeyPair<DCRTPoly> kp;
    auto sk = std::make_shared<PrivateKeyImpl<DCRTPoly>>();
    sk->cc = shared_from_this();
    // the key pair's tag: random (not from the sampling seed), never 0
    {
        std::random_device rd;
        sk->tag = ((uint64_t)rd() << 32 | rd()) | 1;
    }
    s->keyTag = sk->tag;
    std::vector<int64_t> tern(s->n);
    SfheInternal::sampleTernary(s, tern);
    sk->ternary.assign(tern.begin(), tern.end());
    const uint32_t NT = s->tablePrimes();
    sk->s = s->alloc((size_t)NT * s->n);
    const sfp_limbs all{NT, NT, 0};
    sfp_load_i64(s->dev, sk->s->ptr, tern.data(), all);
    sfp_ntt(s->dev, sk->s->ptr, all, 0);
    (void)NP;

    auto pk = std::make_shared<PublicKeyImpl<DCRTPoly>>();
    pk->cc = shared_from_this();
    // rows [q_0..q_L] (+ the q_ext row, prime index extIdx, when ext)
    const uint32_t R = s->Lq + (s->ext ? 1 : 0);
    const sfp_limbs q{R, s->Lq, s->extIdx, 0};
    pk->a = s->alloc((size_t)R * s->n);
    pk->b = s->alloc((size_t)R * s->n);
    sfp_sample_uniform(s->dev, pk->a->ptr, q, s->nextSeed());
    std::vector<int64_t> e(s->n);
    SfheInternal::sampleCBD(s, e);
    sfp_load_i64(s->dev, pk->b->ptr, e.data(), q);
    sfp_ntt(s->dev, pk->b->ptr, q, 0);
    auto t = s->alloc((size_t)R * s->n);
    sfp_mul(s->dev, t->ptr, pk->a->ptr, sk->s->ptr, SfheInternal::Q(s->Lq));
    if (s->ext)
        sfp_mul(s->dev, t->ptr + (size_t)s->Lq * s->n, pk->a->ptr + (size_t)s->Lq * s->n,
                sk->s->ptr + (size_t)s->extIdx * s->n, sfp_limbs{1, 0, s->extIdx, 0});
    sfp_sub(s->dev, pk->b->ptr, pk->b->ptr, t->ptr, q);
    pk->tag = sk->tag;
    kp.publicKey = pk;
    kp.secretKey = sk;
    return kp;
}

void CryptoContextImpl<DCRTPoly>::EvalMultKeyGen(const PrivateKey<DCRTPoly>& sk) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    const uint32_t NP = s->Lq + s->K;
    auto s2 = s->alloc((size_t)NP * s->n);
    sfp_mul(s->dev, s2->ptr, sk->s->ptr, sk->s->ptr, sfp_limbs{NP, NP, 0});
    s->relinKey = SfheInternal::genSwitchKey(this, s2->ptr, sk->s->ptr);
    SfheInternal::genTierKeys(this, s2->ptr, sk->s->ptr, 0);
    s->keyTag = sk->tag;
    // every level's ModUp conversion tables now, as OpenFHE precomputes its
    // CRT tables with the context: built lazily, each upload drained the
    // device inside the first sort
    // (and the fused ModUp's per-level plans with them: built inside the
    // first sort they added ~18 ms of drained uploads to the cold sort)
    for (uint32_t ell = 1; ell <= s->Lq; ++ell)
        sfp_modup_prepare(s->dev, SfheInternal::modupConv(this, ell).data(), ell, s->K, s->alpha);
    if (!s->sharded)
        for (size_t t = 0; t < s->tiers.size(); ++t)
            for (uint32_t ell = 1; ell <= s->tiers[t].maxEll; ++ell)
                sfp_modup_prepare(s->dev, SfheInternal::modupConv(this, ell, (int)t).data(), ell, s->tiers[t].K,
                                  s->alpha);
}

void CryptoContextImpl<DCRTPoly>::EvalRotateKeyGen(const PrivateKey<DCRTPoly>& sk,
                                                   const std::vector<int32_t>& idx,
                                                   const PublicKey<DCRTPoly>&) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    const uint32_t NP = s->Lq + s->K;
    s->keyTag = sk->tag;
    auto sg = s->alloc((size_t)NP * s->n);
    for (int32_t r : idx) {
        s->rotIndices.insert(r);
        uint32_t gal = GaloisForRotation(r);
        if (gal == 1 || s->rotKeys.count(gal)) continue;
        sfp_automorph(s->dev, sg->ptr, sk->s->ptr, gal, sfp_limbs{NP, NP, 0});
        s->rotKeys[gal] = SfheInternal::genSwitchKey(this, sg->ptr, sk->s->ptr);
        SfheInternal::genTierKeys(this, sg->ptr, sk->s->ptr, gal);
    }
}

void CryptoContextImpl<DCRTPoly>::ClearEvalMultKeys() {
    OpLock g(st.get());
    st->relinKey.reset();
    for (auto& t : st->tiers) t.relinKey.reset();
}
void CryptoContextImpl<DCRTPoly>::ClearEvalAutomorphismKeys() {
    OpLock g(st.get());
    st->rotKeys.clear();
    for (auto& t : st->tiers) t.rotKeys.clear();
    st->rotIndices.clear();
}

// ============================================================================
// plaintexts, encryption, decryption

Plaintext CryptoContextImpl<DCRTPoly>::MakeCKKSPackedPlaintext(const std::vector<double>& v,
                                                               uint32_t scaleDeg, uint32_t level,
                                                               const void* params,
                                                               uint32_t slots) const {
    std::vector<std::complex<double>> c(v.begin(), v.end());
    return MakeCKKSPackedPlaintext(c, scaleDeg, level, params, slots);
}

Plaintext CryptoContextImpl<DCRTPoly>::MakeCKKSPackedPlaintext(
    const std::vector<std::complex<double>>& v, uint32_t scaleDeg, uint32_t level, const void*,
    uint32_t slots) const {
    if (scaleDeg != 1) SFHE_THROW("only scale degree 1 plaintexts are supported");
    if (!slots) slots = st->batch;
    if (slots & (slots - 1)) SFHE_THROW("slot count must be a power of two");
    if (slots > st->n / 2) SFHE_THROW("slot count exceeds n/2");
    if (v.size() > slots)
        SFHE_THROW("The size [" + std::to_string(v.size()) +
                   "] of the vector with values should not be greater than slots [" +
                   std::to_string(slots) + "]");
    if (level > st->L) SFHE_THROW("plaintext level exceeds multiplicative depth");
    return std::make_shared<PlaintextImpl>(v, slots, level);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::Encrypt(const PublicKey<DCRTPoly>& pk,
                                                         const Plaintext& pt) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (!pk) SFHE_THROW("null public key");
    if (s->sharded) {  // encrypt every row, keep this rank's
        Ciphertext<DCRTPoly> full;
        {
            FullScope fs(s);
            full = Encrypt(pk, pt);
        }
        return SfheInternal::localize(this, full);
    }
    const uint32_t level = pt->level, ell = s->ellOf(level);
    const sfp_limbs q = st->qmap(ell);
    const uint64_t* m = SfheInternal::encoded(this, pt, level);
    auto ct = SfheInternal::newCt(this, level, pt->slots);
    // FLEXIBLEAUTOEXT: one extra row modulo q_ext (prime index extIdx)
    const uint32_t R = ell + (s->ext ? 1 : 0);
    const sfp_limbs qr{R, ell, s->extIdx, 0};
    const size_t rw = (size_t)R * s->n;
    auto tmp = s->alloc((s->ext ? 5 : 3) * rw);
    uint64_t* v = tmp->ptr;
    uint64_t* e0 = v + rw;
    uint64_t* e1 = e0 + rw;
    std::vector<int64_t> h(s->n);
    SfheInternal::sampleTernary(s, h);
    sfp_load_i64(s->dev, v, h.data(), qr);
    sfp_ntt(s->dev, v, qr, 0);
    SfheInternal::sampleCBD(s, h);
    sfp_load_i64(s->dev, e0, h.data(), qr);
    sfp_ntt(s->dev, e0, qr, 0);
    SfheInternal::sampleCBD(s, h);
    sfp_load_i64(s->dev, e1, h.data(), qr);
    sfp_ntt(s->dev, e1, qr, 0);
    if (!s->ext) {
        sfp_mul_add(s->dev, ct->c0, v, pk->b->ptr, e0, q);
        sfp_add(s->dev, ct->c0, ct->c0, m, q);
        sfp_mul_add(s->dev, ct->c1, v, pk->a->ptr, e1, q);
        return SfheInternal::traced(this, ct, "Encrypt");
    }
    // (v*pk + (e0 + q_ext*m, e1)) mod Q*q_ext; the q_ext row of q_ext*m is 0.
    // Dividing by q_ext leaves m at scale Delta_level with the encryption
    // noise shrunk by q_ext (only the rounding of the division remains).
    uint64_t* c0x = e1 + rw;
    uint64_t* c1x = c0x + rw;
    const size_t qw = (size_t)ell * s->n, pkExt = (size_t)s->Lq * s->n;
    const sfp_limbs x1{1, 0, s->extIdx, 0};
    sfp_mul_add(s->dev, c0x, v, pk->b->ptr, e0, q);
    sfp_mul_const(s->dev, c1x, m, s->extModQ.data(), q);
    sfp_add(s->dev, c0x, c0x, c1x, q);
    sfp_mul_add(s->dev, c1x, v, pk->a->ptr, e1, q);
    sfp_mul_add(s->dev, c0x + qw, v + qw, pk->b->ptr + pkExt, e0 + qw, x1);
    sfp_mul_add(s->dev, c1x + qw, v + qw, pk->a->ptr + pkExt, e1 + qw, x1);
    sfp_rescale_ext(s->dev, ct->c0, c0x, R, s->extIdx, s->extInvModQ.data(), 2, rw,
                    (size_t)(ct->c1 - ct->c0));
    return SfheInternal::traced(this, ct, "Encrypt");
}

void CryptoContextImpl<DCRTPoly>::Decrypt(const PrivateKey<DCRTPoly>& sk,
                                          const Ciphertext<DCRTPoly>& ct, Plaintext* out) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&ct});
    SfheContextState* s = st.get();
    if (!sk) SFHE_THROW("null secret key");
    if (s->sharded) {  // every rank gathers the rows and decrypts
        auto full = SfheInternal::gatherFull(s, ct);
        FullScope fs(s);
        auto fc = std::make_shared<CiphertextImpl<DCRTPoly>>(*ct);
        fc->buf = full;
        fc->c0 = full->ptr;
        fc->c1 = fc->c0 + (size_t)s->ellOf(ct->level) * s->n;
        return Decrypt(sk, fc, out);
    }
    const uint32_t ell = s->ellOf(ct->level);
    const uint32_t nl = std::min<uint32_t>(2, ell);
    const sfp_limbs q = SfheInternal::Q(nl);
    auto t = s->alloc((size_t)nl * s->n);
    sfp_mul_add(s->dev, t->ptr, ct->c1, sk->s->ptr, ct->c0, q);
    sfp_ntt(s->dev, t->ptr, q, 1);
    std::vector<u64> h((size_t)nl * s->n);
    sfp_d2h(s->dev, h.data(), t->ptr, h.size() * 8);
    const char* err = sfp_last_error(s->dev);
    if (err) SFHE_THROW(std::string("device error: ") + err);
    std::vector<double> c(s->n);
    const u64 q0 = s->primes[0];
    // the decoder reads coefficients i*gap and n/2 + i*gap only (sparse
    // packing): reconstruct just those (all of them when slots = n/2)
    const uint32_t gap = (s->n / 2) / std::max<uint32_t>(1, ct->slots);
    auto each = [&](auto&& f) {
        for (uint32_t j = 0; j < s->n / 2; j += gap) {
            f(j);
            f(s->n / 2 + j);
        }
    };
    if (nl == 1) {
        each([&](uint32_t i) {
            u64 x = h[i];
            double v = x > q0 / 2 ? -(double)(q0 - x) : (double)x;
            c[i] = v / ct->scale;
        });
    } else {
        const u64 q1 = s->primes[1];
        const u64 q0inv = invmod(q0 % q1, q1);
        const u64 q0invS = (u64)(((u128)q0inv << 64) / q1);  // Shoup companion
        const u128 Q = (u128)q0 * q1;
        each([&](uint32_t i) {
            const u64 a0 = h[i], a1 = h[s->n + i];
            const u64 r0 = a0 % q1;
            const u64 d = a1 >= r0 ? a1 - r0 : a1 + q1 - r0;
            u64 m = d * q0inv - (u64)(((u128)d * q0invS) >> 64) * q1;  // d * q0^-1 mod q1, in [0, 2 q1)
            if (m >= q1) m -= q1;
            u128 x = (u128)a0 + (u128)q0 * m;
            double v = x > Q / 2 ? -(double)(Q - x) : (double)x;
            c[i] = v / ct->scale;
        });
    }
    std::vector<std::complex<double>> vals;
    ckks_decode(c, ct->slots, s->n, vals);
    auto pt = std::make_shared<PlaintextImpl>(vals, ct->slots, ct->level);
    // precision estimate from the imaginary parts (inputs are real)
    double var = 0;
    for (auto& z : vals) var += z.imag() * z.imag();
    double sd = std::sqrt(var / std::max<size_t>(1, vals.size()));
    pt->logError = sd > 0 ? std::log2(sd) : -60.0;
    pt->logPrecision = -pt->logError;
    *out = pt;
}

const std::vector<double>& PlaintextImpl::GetRealPackedValue() const {
    realCache.resize(std::min(length, values.size()));
    for (size_t i = 0; i < realCache.size(); ++i) realCache[i] = values[i].real();
    return realCache;
}

std::ostream& operator<<(std::ostream& os, const Plaintext& pt) {
    const auto& v = pt->GetRealPackedValue();
    os << "(";
    for (size_t i = 0; i < v.size(); ++i) os << v[i] << (i + 1 < v.size() ? ", " : "");
    return os << " ... )";
}

Ciphertext<DCRTPoly> CiphertextImpl<DCRTPoly>::Clone() const {
    OpLock g(cc->state());
    // a deferred product is computed first (unrescaled while rescaling is
    // lazy: the copy's consumer decides); pending rows are copied as they are
    if (def)
        SfheInternal::materialize(const_cast<CiphertextImpl<DCRTPoly>&>(*this),
                                  SfheInternal::lazy(cc->state()));
    cc->state()->dep(buf.get());
    auto self = std::make_shared<CiphertextImpl<DCRTPoly>>(*this);
    return SfheInternal::copyOf(cc.get(), self);
}

uint32_t CiphertextImpl<DCRTPoly>::GetNumLimbs() const { return cc->state()->ellOf(level); }

// ============================================================================
// evaluator: additive

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalAdd(const Ciphertext<DCRTPoly>& a0,
                                                         const Ciphertext<DCRTPoly>& b0) {
    OpLock g(st.get());
    if (auto r = SfheInternal::lazyAdd(this, a0, b0, false)) return SfheInternal::traced(this, r, "EvalAdd");
    SfheInternal::deps(st.get(), {&a0, &b0});
    auto a = a0, b = b0;
    SfheInternal::align(this, a, b);
    auto out = SfheInternal::newCt(this, a->level, std::max(a->slots, b->slots));
    const uint32_t ell = st->ellOf(a->level);
    if (SfheInternal::packed(st.get(), {out->c0, a->c0, b->c0}, {out->c1, a->c1, b->c1}, a->level)) {
        sfp_add(st->dev, out->c0, a->c0, b->c0, SfheInternal::both(st.get(), ell));
    } else {
        sfp_add(st->dev, out->c0, a->c0, b->c0, st->qmap(ell));
        sfp_add(st->dev, out->c1, a->c1, b->c1, st->qmap(ell));
    }
    st->stats.add++;
    st->countBytes(6.0 * ell * st->n * 8);
    return SfheInternal::traced(this, out, "EvalAdd");
}

void CryptoContextImpl<DCRTPoly>::EvalAddInPlace(Ciphertext<DCRTPoly>& a,
                                                 const Ciphertext<DCRTPoly>& b0) {
    OpLock g(st.get());
    if (SfheInternal::isLazy(a) || SfheInternal::isLazy(b0)) {
        a = EvalAdd(a, b0);
        return;
    }
    SfheInternal::deps(st.get(), {&a, &b0});
    auto b = b0;
    // in place only on an exclusively owned buffer
    if (a->level != b->level || a->buf.use_count() > 1 ||
        a->c1 - a->c0 != (ptrdiff_t)st->polyWords(a->level)) {
        a = EvalAdd(a, b);
        return;
    }
    const uint32_t ell = st->ellOf(a->level);
    if (SfheInternal::packed(st.get(), {a->c0, b->c0}, {a->c1, b->c1}, a->level)) {
        sfp_add(st->dev, a->c0, a->c0, b->c0, SfheInternal::both(st.get(), ell));
    } else {
        sfp_add(st->dev, a->c0, a->c0, b->c0, st->qmap(ell));
        sfp_add(st->dev, a->c1, a->c1, b->c1, st->qmap(ell));
    }
    st->wrote(a->buf.get());
    a->slots = std::max(a->slots, b->slots);
    st->stats.add++;
    st->countBytes(6.0 * ell * st->n * 8);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalAdd(const Ciphertext<DCRTPoly>& a,
                                                         double c) {
    OpLock g(st.get());
    if (a->pend && !a->def) {  // unrescaled rows: the constant at the product's scale
        st->dep(a->buf.get());
        const uint32_t ell = st->ellOf(a->level) + 1;
        auto out = SfheInternal::newPendingCt(this, a->level, a->slots);
        auto k = SfheInternal::constResidues(st.get(), c * a->scale, ell);
        if (2 * k.size() <= SFP_MAX_LIMBS &&
            SfheInternal::packed(st.get(), {out->c0, a->c0}, {out->c1, a->c1}, a->level - 1)) {
            k.resize(2 * k.size(), 0);  // c1 rows: + 0, i.e. the copy, in the same launch
            sfp_add_const(st->dev, out->c0, a->c0, k.data(), SfheInternal::both(st.get(), ell));
        } else {
            sfp_add_const(st->dev, out->c0, a->c0, k.data(), st->qmap(ell));
            sfp_d2d(st->dev, out->c1, a->c1, (size_t)st->rows(ell) * st->n * 8);
        }
        st->stats.add++;
        st->countBytes(4.0 * ell * st->n * 8);
        return SfheInternal::traced(this, out, "EvalAdd");
    }
    SfheInternal::deps(st.get(), {&a});
    const uint32_t ell = st->ellOf(a->level);
    auto out = SfheInternal::newCt(this, a->level, a->slots);
    auto k = SfheInternal::constResidues(st.get(), c * a->scale, ell);
    if (2 * k.size() <= SFP_MAX_LIMBS &&
        SfheInternal::packed(st.get(), {out->c0, a->c0}, {out->c1, a->c1}, a->level)) {
        k.resize(2 * k.size(), 0);  // c1 rows: + 0, i.e. the copy, in the same launch
        sfp_add_const(st->dev, out->c0, a->c0, k.data(), SfheInternal::both(st.get(), ell));
    } else {
        sfp_add_const(st->dev, out->c0, a->c0, k.data(), st->qmap(ell));
        sfp_d2d(st->dev, out->c1, a->c1, st->polyWords(a->level) * 8);
    }
    st->stats.add++;
    st->countBytes(4.0 * ell * st->n * 8);
    return SfheInternal::traced(this, out, "EvalAdd");
}

void CryptoContextImpl<DCRTPoly>::EvalAddInPlace(Ciphertext<DCRTPoly>& a, double c) {
    a = EvalAdd(a, c);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalAdd(const Ciphertext<DCRTPoly>& a,
                                                         const Plaintext& p) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    const uint32_t ell = st->ellOf(a->level);
    const uint64_t* m = SfheInternal::encoded(this, p, a->level);
    auto out = SfheInternal::newCt(this, a->level, std::max(a->slots, p->slots));
    sfp_add(st->dev, out->c0, a->c0, m, st->qmap(ell));
    sfp_d2d(st->dev, out->c1, a->c1, st->polyWords(a->level) * 8);
    st->stats.add++;
    st->countBytes(5.0 * ell * st->n * 8);
    return SfheInternal::traced(this, out, "EvalAdd");
}

void CryptoContextImpl<DCRTPoly>::EvalAddInPlace(Ciphertext<DCRTPoly>& a, const Plaintext& p) {
    a = EvalAdd(a, p);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalSub(const Ciphertext<DCRTPoly>& a0,
                                                         const Ciphertext<DCRTPoly>& b0) {
    OpLock g(st.get());
    if (auto r = SfheInternal::lazyAdd(this, a0, b0, true)) return SfheInternal::traced(this, r, "EvalSub");
    SfheInternal::deps(st.get(), {&a0, &b0});
    auto a = a0, b = b0;
    SfheInternal::align(this, a, b);
    auto out = SfheInternal::newCt(this, a->level, std::max(a->slots, b->slots));
    const uint32_t ell = st->ellOf(a->level);
    if (SfheInternal::packed(st.get(), {out->c0, a->c0, b->c0}, {out->c1, a->c1, b->c1}, a->level)) {
        sfp_sub(st->dev, out->c0, a->c0, b->c0, SfheInternal::both(st.get(), ell));
    } else {
        sfp_sub(st->dev, out->c0, a->c0, b->c0, st->qmap(ell));
        sfp_sub(st->dev, out->c1, a->c1, b->c1, st->qmap(ell));
    }
    st->stats.add++;
    st->countBytes(6.0 * ell * st->n * 8);
    return SfheInternal::traced(this, out, "EvalSub");
}

void CryptoContextImpl<DCRTPoly>::EvalSubInPlace(Ciphertext<DCRTPoly>& a,
                                                 const Ciphertext<DCRTPoly>& b) {
    a = EvalSub(a, b);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalNegate(const Ciphertext<DCRTPoly>& a) {
    OpLock g(st.get());
    if (a->pend && !a->def) {
        st->dep(a->buf.get());
        const uint32_t ell = st->ellOf(a->level) + 1;
        auto out = SfheInternal::newPendingCt(this, a->level, a->slots);
        sfp_neg(st->dev, out->c0, a->c0, st->qmap(ell));
        sfp_neg(st->dev, out->c1, a->c1, st->qmap(ell));
        st->countBytes(4.0 * ell * st->n * 8);
        return SfheInternal::traced(this, out, "EvalNegate");
    }
    SfheInternal::deps(st.get(), {&a});
    const uint32_t ell = st->ellOf(a->level);
    auto out = SfheInternal::newCt(this, a->level, a->slots);
    if (SfheInternal::packed(st.get(), {out->c0, a->c0}, {out->c1, a->c1}, a->level)) {
        sfp_neg(st->dev, out->c0, a->c0, SfheInternal::both(st.get(), ell));
    } else {
        sfp_neg(st->dev, out->c0, a->c0, st->qmap(ell));
        sfp_neg(st->dev, out->c1, a->c1, st->qmap(ell));
    }
    st->countBytes(4.0 * ell * st->n * 8);
    return SfheInternal::traced(this, out, "EvalNegate");
}

void CryptoContextImpl<DCRTPoly>::EvalNegateInPlace(Ciphertext<DCRTPoly>& a) { a = EvalNegate(a); }

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalSub(double c, const Ciphertext<DCRTPoly>& a) {
    return EvalAdd(EvalNegate(a), c);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalSub(const Ciphertext<DCRTPoly>& a,
                                                         const Plaintext& p) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    const uint32_t ell = st->ellOf(a->level);
    const uint64_t* m = SfheInternal::encoded(this, p, a->level);
    auto out = SfheInternal::newCt(this, a->level, std::max(a->slots, p->slots));
    sfp_sub(st->dev, out->c0, a->c0, m, st->qmap(ell));
    sfp_d2d(st->dev, out->c1, a->c1, st->polyWords(a->level) * 8);
    st->stats.add++;
    st->countBytes(5.0 * ell * st->n * 8);
    return SfheInternal::traced(this, out, "EvalSub");
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalSub(const Plaintext& p,
                                                         const Ciphertext<DCRTPoly>& a) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    const uint32_t ell = st->ellOf(a->level);
    const uint64_t* m = SfheInternal::encoded(this, p, a->level);
    auto out = SfheInternal::newCt(this, a->level, std::max(a->slots, p->slots));
    sfp_sub(st->dev, out->c0, m, a->c0, st->qmap(ell));
    sfp_neg(st->dev, out->c1, a->c1, st->qmap(ell));
    st->stats.add++;
    st->countBytes(5.0 * ell * st->n * 8);
    return SfheInternal::traced(this, out, "EvalSub");
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalAddMany(
    const std::vector<Ciphertext<DCRTPoly>>& v) {
    if (v.empty()) SFHE_THROW("EvalAddMany of an empty vector");
    OpLock g(st.get());
    std::vector<Ciphertext<DCRTPoly>> cur(v.begin(), v.end());
    while (cur.size() > 1) {
        std::vector<Ciphertext<DCRTPoly>> nxt;
        for (size_t i = 0; i + 1 < cur.size(); i += 2) nxt.push_back(EvalAdd(cur[i], cur[i + 1]));
        if (cur.size() & 1) nxt.push_back(cur.back());
        cur.swap(nxt);
    }
    return cur[0]->buf.use_count() > 1 && cur[0] == v[0] ? cur[0]->Clone() : cur[0];
}

// ============================================================================
// evaluator: multiplicative

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalMult(const Ciphertext<DCRTPoly>& a,
                                                          double c) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    SfheContextState* s = st.get();
    const uint32_t ell = s->ellOf(a->level);
    if (ell < 2) SFHE_THROW("no levels left (multiplicative depth exhausted)");
    // integer K with scale_a * K / q_last = Delta_{l+1} * c
    double K = c * s->scale[a->level + 1] * (double)s->primes[ell - 1] / a->scale;
    auto k = SfheInternal::constResidues(s, K, ell);
    s->stats.constmult++;
    s->countBytes(4.0 * ell * s->n * 8);
    if (SfheInternal::lazy(s)) {
        auto op = std::make_shared<DeferredConstMult>();
        op->pin = a->buf;
        op->c0 = a->c0;
        op->c1 = a->c1;
        op->level = a->level;
        op->slots = a->slots;
        op->scale = a->scale;
        op->k = std::move(k);
        return SfheInternal::deferredCt(this, a->level + 1, a->slots, op);
    }
    return SfheInternal::traced(this, SfheInternal::mulRescale(this, a, a->level, k.data(), nullptr, a->slots),
                                "EvalMult");
}

void CryptoContextImpl<DCRTPoly>::EvalMultInPlace(Ciphertext<DCRTPoly>& a, double c) {
    a = EvalMult(a, c);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalMult(const Ciphertext<DCRTPoly>& a,
                                                          const Plaintext& p) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    SfheContextState* s = st.get();
    const uint32_t ell = s->ellOf(a->level);
    if (ell < 2) SFHE_THROW("no levels left (multiplicative depth exhausted)");
    s->stats.ptmult++;
    s->countBytes(5.0 * ell * s->n * 8);
    if (SfheInternal::lazy(s)) {
        auto op = std::make_shared<DeferredPlainMult>();
        op->pin = a->buf;
        op->c0 = a->c0;
        op->c1 = a->c1;
        op->level = a->level;
        op->slots = std::max(a->slots, p->slots);
        op->scale = a->scale;
        op->pt = p;
        return SfheInternal::deferredCt(this, a->level + 1, op->slots, op);
    }
    const uint64_t* m = SfheInternal::encoded(this, p, a->level);
    return SfheInternal::traced(
        this, SfheInternal::mulRescale(this, a, a->level, nullptr, m, std::max(a->slots, p->slots)), "EvalMult");
}

void CryptoContextImpl<DCRTPoly>::EvalMultInPlace(Ciphertext<DCRTPoly>& a, const Plaintext& p) {
    a = EvalMult(a, p);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalMult(const Ciphertext<DCRTPoly>& a0,
                                                          const Ciphertext<DCRTPoly>& b0) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a0, &b0});
    SfheContextState* s = st.get();
    if (!s->relinKey) SFHE_THROW("EvalMultKeyGen must be called before EvalMult");
    auto a = a0, b = b0;
    SfheInternal::align(this, a, b);
    const uint32_t ell = s->ellOf(a->level);
    if (ell < 2) SFHE_THROW("no levels left (multiplicative depth exhausted)");
    const size_t pw = s->polyWords(a->level);
    s->stats.tensor++;
    s->countBytes(7.0 * ell * s->n * 8);
    const uint32_t slots = std::max(a->slots, b->slots);
    if (SfheInternal::lazy(s) && SfheInternal::fusedRescale()) {
        auto op = std::make_shared<DeferredRelin>();
        op->pa = a->buf;
        op->pb = b->buf;
        op->a0 = a->c0;
        op->a1 = a->c1;
        op->b0 = b->c0;
        op->b1 = b->c1;
        op->level = a->level;
        op->slots = slots;
        return SfheInternal::deferredCt(this, a->level + 1, slots, op);
    }
    if (SfheInternal::fusedRescale())
        return SfheInternal::traced(
            this, SfheInternal::multRelinRescale(this, a->c0, a->c1, b->c0, b->c1, a->level, slots), "EvalMult");
    auto t = s->alloc(3 * pw);
    uint64_t* d0 = t->ptr;
    uint64_t* d1 = d0 + pw;
    uint64_t* d2 = d1 + pw;
    sfp_tensor(s->dev, d0, d1, d2, a->c0, a->c1, b->c0, b->c1, st->qmap(ell));
    SfheInternal::keySwitch(this, d2, ell, s->relinFor(ell), d0, d1, 1, 1);
    return SfheInternal::traced(this, SfheInternal::rescale(this, d0, d1, a->level, slots), "EvalMult");
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalSquare(const Ciphertext<DCRTPoly>& a) {
    return EvalMult(a, a);
}

std::vector<Ciphertext<DCRTPoly>> CryptoContextImpl<DCRTPoly>::EvalMultMany(
    const std::vector<Ciphertext<DCRTPoly>>& a0, const std::vector<Ciphertext<DCRTPoly>>& b0) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (a0.size() != b0.size()) SFHE_THROW("operand count mismatch");
    const size_t cnt = a0.size();
    std::vector<Ciphertext<DCRTPoly>> out(cnt);
    // the products are formed canonically (as a deferred product is when its
    // consumer needs the canonical form: the same values); for consumers that
    // would take a lazy product's pending rows, use EvalMult
    if (cnt < 2 || !SfheInternal::fusedRescale()) {
        for (size_t i = 0; i < cnt; ++i) out[i] = EvalMult(a0[i], b0[i]);
        return out;
    }
    if (!s->relinKey) SFHE_THROW("EvalMultKeyGen must be called before EvalMult");
    std::vector<Ciphertext<DCRTPoly>> A(a0), B(b0);
    for (size_t i = 0; i < cnt; ++i) {
        SfheInternal::deps(s, {&a0[i], &b0[i]});
        SfheInternal::align(this, A[i], B[i]);
        if (s->ellOf(A[i]->level) < 2) SFHE_THROW("no levels left (multiplicative depth exhausted)");
        s->stats.tensor++;
        s->countBytes(7.0 * s->ellOf(A[i]->level) * s->n * 8);
    }
    // runs of up to SFP_BATCH_MAX consecutive pairs at one level
    for (size_t i = 0; i < cnt;) {
        size_t j = i + 1;
        while (j < cnt && j - i < batchWidth() && A[j]->level == A[i]->level) ++j;
        std::vector<const CiphertextImpl<DCRTPoly>*> pa, pb;
        std::vector<uint32_t> slots;
        for (size_t k = i; k < j; ++k) {
            pa.push_back(A[k].get());
            pb.push_back(B[k].get());
            slots.push_back(std::max(A[k]->slots, B[k]->slots));
        }
        auto r = SfheInternal::multRelinRescaleMany(this, pa, pb, A[i]->level, slots);
        for (size_t k = i; k < j; ++k) out[k] = SfheInternal::traced(this, r[k - i], "EvalMult");
        i = j;
    }
    return out;
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalMultAddPlain(
    const std::vector<Ciphertext<DCRTPoly>>& a, const std::vector<Plaintext>& p) {
    OpLock g(st.get());
    SfheInternal::depsv(st.get(), a);
    SfheContextState* s = st.get();
    if (a.empty() || a.size() != p.size()) SFHE_THROW("operand count mismatch");
    uint32_t level = 0, slots = 0;
    for (size_t i = 0; i < a.size(); ++i) {
        level = std::max(level, a[i]->level);
        slots = std::max(slots, std::max(a[i]->slots, p[i]->slots));
    }
    const uint32_t ell = s->ellOf(level);
    if (ell < 2) SFHE_THROW("no levels left (multiplicative depth exhausted)");
    std::vector<Ciphertext<DCRTPoly>> al(a.size());
    std::vector<const uint64_t*> x0, x1, m;
    for (size_t i = 0; i < a.size(); ++i) {
        al[i] = SfheInternal::adjust(this, a[i], level);
        x0.push_back(al[i]->c0);
        x1.push_back(al[i]->c1);
    }
    s->stats.ptmult += a.size();
    if (SfheInternal::lazy(s)) {
        auto op = std::make_shared<DeferredMacPlain>();
        for (auto& c : al) op->pins.push_back(c->buf);
        op->x0 = x0;
        op->x1 = x1;
        op->pts = p;
        op->level = level;
        op->slots = slots;
        s->countBytes((3.0 * a.size() + 2.0) * ell * s->n * 8);
        return SfheInternal::deferredCt(this, level + 1, slots, op);
    }
    SfheInternal::encodeBatch(this, p, level);
    for (size_t i = 0; i < a.size(); ++i) m.push_back(SfheInternal::encoded(this, p[i], level));
    const size_t pw = s->polyWords(level);
    auto tmp = s->alloc(2 * pw);
    uint64_t* t0 = tmp->ptr;
    uint64_t* t1 = t0 + pw;
    for (size_t done = 0; done < a.size(); done += SFP_MAX_WSUM) {
        uint32_t take = (uint32_t)std::min<size_t>(SFP_MAX_WSUM, a.size() - done);
        if (done == 0) {
            sfp_mac_plain2(s->dev, t0, t1, x0.data(), x1.data(), m.data(), take, st->qmap(ell));
        } else {
            auto part = s->alloc(2 * pw);
            sfp_mac_plain2(s->dev, part->ptr, part->ptr + pw, x0.data() + done, x1.data() + done,
                           m.data() + done, take, st->qmap(ell));
            sfp_add(s->dev, t0, t0, part->ptr, st->qmap(ell));
            sfp_add(s->dev, t1, t1, part->ptr + pw, st->qmap(ell));
        }
    }
    s->countBytes((3.0 * a.size() + 2.0) * ell * s->n * 8);
    return SfheInternal::traced(this, SfheInternal::rescale(this, t0, t1, level, slots), "EvalMultAddPlain");
}

// ============================================================================
// rotations

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalRotate(const Ciphertext<DCRTPoly>& a,
                                                            int32_t r) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (!(SfheInternal::lazy(s) && SfheInternal::isLazy(a))) SfheInternal::deps(s, {&a});
    uint32_t gal = GaloisForRotation(r);
    if (gal == 1) return a->Clone();
    if (!s->rotKeys.count(gal))
        SFHE_THROW("EvalKey for index [" + std::to_string(gal) + "] (rotation " +
                   std::to_string(r) + ") is not found");
    // a lazy product rotates before its rescale: the key switch's rounding is
    // then divided by the prime the settling rescale drops
    const bool pend = SfheInternal::lazy(s) && SfheInternal::isLazy(a);
    if (pend) {
        SfheInternal::materialize(*a, true);
        s->dep(a->buf.get());
    }
    const uint32_t ell = SfheInternal::ctEll(s, *a);
    auto out = pend ? SfheInternal::newPendingCt(this, a->level, a->slots) : SfheInternal::newCt(this, a->level, a->slots);
    auto t = s->alloc((size_t)s->rows(ell) * s->n);
    sfp_automorph(s->dev, out->c0, a->c0, gal, st->qmap(ell));
    sfp_automorph(s->dev, t->ptr, a->c1, gal, st->qmap(ell));
    s->stats.automorph++;
    s->countBytes(3.0 * ell * s->n * 8);
    // c0' = sigma(c0) + ks0, c1' = ks1 (with the key of ell's special-prime tier)
    SfheInternal::keySwitch(this, t->ptr, ell, *s->rotFor(gal, ell), out->c0, out->c1, 1, 0);
    return SfheInternal::traced(this, out, "EvalRotate");
}

std::shared_ptr<FastRotationPrecomp> CryptoContextImpl<DCRTPoly>::EvalFastRotationPrecompute(
    const Ciphertext<DCRTPoly>& a) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    // Pending rows are rotated as they are (see EvalRotate).  A deferred
    // product is computed in canonical form first: its hoisted rotations
    // feed plaintext products (the blind rotations), which would otherwise
    // settle every rotated copy separately.
    const bool pend = SfheInternal::lazy(s) && a->pend && !a->def;
    if (pend) {
        SfheInternal::materialize(*a, true);
        s->dep(a->buf.get());
    } else {
        SfheInternal::deps(s, {&a});
    }
    auto pre = std::make_shared<FastRotationPrecomp>();
    const uint32_t ell = SfheInternal::ctEll(s, *a);
    pre->level = a->level;
    pre->pend = pend;
    pre->beta = (ell + s->alpha - 1) / s->alpha;
    if (pend) {
        pre->pinBuf = a->buf;
        pre->pinC0 = a->c0;
    }
    if (s->shardAt(ell)) {
        pre->stride = (size_t)s->extmap(ell).count * s->n;
        pre->ext = s->alloc(pre->stride * pre->beta);
        SfheInternal::modupShard(s, pre->ext->ptr, a->c1, ell);
        return pre;
    }
    // the extended digits over ell's special-prime tier (its rotation keys
    // exist for every rotation key: they are generated together)
    const int tier = s->tierAt(ell);
    const uint32_t K = s->Kof(tier);
    pre->stride = (size_t)(ell + K) * s->n;
    pre->ext = s->alloc(pre->stride * pre->beta);
    auto scratch = s->alloc((size_t)ell * s->n);
    auto& convs = SfheInternal::modupConv(this, ell, tier);
    sfp_modup(s->dev, pre->ext->ptr, a->c1, ell, K, s->Lq, s->alpha, convs.data(), scratch->ptr);
    return pre;
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalFastRotation(
    const Ciphertext<DCRTPoly>& a, int32_t r, uint32_t, const std::shared_ptr<FastRotationPrecomp>& pre) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    // A pending precomputation rotates the unrescaled rows it pinned (the
    // shared ciphertext may have been settled since: same value, other form).
    const bool pinned = pre && pre->pend;
    if (pinned) {
        s->dep(pre->pinBuf.get());
    } else {
        SfheInternal::deps(s, {&a});
    }
    uint32_t gal = GaloisForRotation(r);
    if (gal == 1) return a->Clone();
    if (!pre || pre->level != a->level)
        SFHE_THROW("fast-rotation precomputation does not match");
    if (!s->rotKeys.count(gal)) SFHE_THROW("EvalKey for rotation " + std::to_string(r) + " is not found");
    const uint32_t ell = pinned ? s->ellOf(pre->level) + 1 : SfheInternal::ctEll(s, *a);
    // the key of the precomputation's tier (its extended rows: ell + K' per digit)
    const DeviceBufferPtr* key = s->rotFor(gal, ell);
    if (!s->shardAt(ell) && (size_t)(ell + s->Kof((*key)->ksTier)) * s->n != pre->stride)
        key = &s->rotKeys.at(gal);
    const uint64_t* c0in = pinned ? pre->pinC0 : a->c0;
    // sigma commutes with the (coefficient-wise) base extension, so rotating
    // the extended digits equals extending the rotated c1.  Unsharded, the
    // inner product reads the shared digits through sigma (sfp_ks_inner_aut:
    // the permuted copy is never written); SFHE_KS_AUT=0 permutes them first.
    static const bool autFused = [] {
        const char* v = std::getenv("SFHE_KS_AUT");
        return !v || *v != '0';
    }();
    const bool fuse = autFused && !s->shardAt(ell);
    DeviceBufferPtr ext;
    if (!fuse) {
        ext = s->alloc(pre->stride * pre->beta);
        // one permutation launch over every digit's rows (the map is prime-independent)
        const uint32_t rows = pre->beta * (uint32_t)(pre->stride / s->n);
        sfp_automorph(s->dev, ext->ptr, pre->ext->ptr, gal, sfp_limbs{rows, rows, 0, 0});
    } else {
        s->dep(pre->ext.get());
    }
    auto out = pre->pend ? SfheInternal::newPendingCt(this, a->level, a->slots)
                         : SfheInternal::newCt(this, a->level, a->slots);
    sfp_automorph(s->dev, out->c0, c0in, gal, st->qmap(ell));
    SfheInternal::innerAndModDown(this, fuse ? pre->ext->ptr : ext->ptr, pre->stride, pre->beta, ell, *key, out->c0,
                                  out->c1, 1, 0, fuse ? gal : 0u);
    s->stats.keyswitch++;
    s->stats.automorph++;
    s->countBytes((3.0 * ell + 2.0 * pre->beta * (pre->stride / s->n)) * s->n * 8);
    return SfheInternal::traced(this, out, "EvalFastRotation");
}

// Output aggregation: the terms' key switches share the accumulator in the
// extended basis (sfp_ks_inner_acc) and one ModDown, so a sum of R rotations
// costs R ModUps and one ModDown instead of R of each.  Terms with a rotation
// of a multiple of the slot count are added as they are.  SFHE_ROTSUM=0
// (diagnostic) sums individual EvalRotates.
Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalRotateSum(const std::vector<Ciphertext<DCRTPoly>>& a,
                                                                const std::vector<int32_t>& r) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (a.empty()) return EvalAddMany(a);  // the reference's error for an empty sum
    if (a.size() != r.size()) SFHE_THROW("EvalRotateSum: operand count mismatch");
    static const bool off = [] {
        const char* v = std::getenv("SFHE_ROTSUM");
        return v && *v == '0';
    }();
    std::vector<size_t> rot, ident;
    for (size_t k = 0; k < a.size(); ++k) (GaloisForRotation(r[k]) == 1 ? ident : rot).push_back(k);
    const bool pend = !rot.empty() && SfheInternal::lazy(s) && SfheInternal::isLazy(a[rot[0]]);
    bool agg = !off && rot.size() >= 2;
    for (size_t k : rot)
        agg = agg && a[k]->level == a[rot[0]]->level &&
              (SfheInternal::lazy(s) && SfheInternal::isLazy(a[k])) == pend;
    if (!agg) {
        std::vector<Ciphertext<DCRTPoly>> terms;
        for (size_t k = 0; k < a.size(); ++k) terms.push_back(EvalRotate(a[k], r[k]));
        return EvalAddMany(terms);
    }
    for (size_t k : rot)
        if (!s->rotKeys.count(GaloisForRotation(r[k])))
            SFHE_THROW("EvalKey for rotation " + std::to_string(r[k]) + " is not found");
    // pending products rotate before their rescale, as in EvalRotate
    uint32_t slots = 0;
    if (pend) macGroups(this, a, rot);
    for (size_t k : rot) {
        if (pend) {
            SfheInternal::materialize(*a[k], true);
            s->dep(a[k]->buf.get());
        } else {
            SfheInternal::deps(s, {&a[k]});
        }
        slots = std::max(slots, a[k]->slots);
    }
    const uint32_t level = a[rot[0]]->level, ell = SfheInternal::ctEll(s, *a[rot[0]]);
    // the terms' keys of their (shared) limb count's special-prime tier
    std::vector<const DeviceBufferPtr*> keys;
    for (size_t k : rot) keys.push_back(s->rotFor(GaloisForRotation(r[k]), ell));
    const int tier = (*keys[0])->ksTier;
    for (auto* k : keys)
        if ((*k)->ksTier != tier) SFHE_THROW("internal: rotation keys of different special-prime tiers");
    const uint32_t n = s->n, K = s->Kof(tier), beta = (ell + s->alpha - 1) / s->alpha;
    const bool shard = s->shardAt(ell);  // local rows; the exchanges inside modupShard / modDownShard
    const size_t stride = (size_t)(shard ? s->extmap(ell).count : ell + K) * n;
    auto out = pend ? SfheInternal::newPendingCt(this, level, slots) : SfheInternal::newCt(this, level, slots);
    auto acc = s->alloc(2 * stride);
    int rowDone = 0;
    auto& convs = SfheInternal::modupConv(this, ell, tier);
    if (!shard && sfp_modup_inner_phase(s->dev, nullptr, nullptr, nullptr, ell, K, s->Lq, s->alpha, convs.data(),
                                        nullptr, nullptr, nullptr, 0, 0, 0, nullptr, nullptr, 0) == 0) {
        // The terms' rotations and ModUps are independent: each chunk of
        // them runs as batched ops (merged launches), then its terms' fused
        // inner products accumulate into acc in turn (never merged: one
        // accumulator), the last one with the ModDown's first inverse pass.
        const size_t w = batchWidth();
        // sigma_k(c0_k) of every term but the first, summed into out->c0 by one
        // weighted sum (weights 1) after the loop instead of one add per term
        std::vector<DeviceBufferPtr> c0s;
        static const bool oneSumOn = [] {  // SFHE_ROTSUM_C0=0: one add per term (A/B)
            const char* v = std::getenv("SFHE_ROTSUM_C0");
            return !v || *v != '0';
        }();
        const bool oneSum = oneSumOn && rot.size() <= SFP_MAX_WSUM;
        for (size_t b0 = 0; b0 < rot.size(); b0 += w) {
            const size_t b1 = std::min(rot.size(), b0 + w);
            std::vector<DeviceBufferPtr> tb, cb, eb, sb;
            {
                BatchScope bs(this, (uint32_t)(b1 - b0));
                for (size_t i = b0; i < b1; ++i) {
                    bs.lane((uint32_t)(i - b0));
                    const Ciphertext<DCRTPoly>& x = a[rot[i]];
                    const uint32_t gal = GaloisForRotation(r[rot[i]]);
                    tb.push_back(s->alloc((size_t)ell * n));
                    eb.push_back(s->alloc(stride * beta));
                    sb.push_back(s->alloc((size_t)ell * n));
                    cb.push_back(i ? s->alloc((size_t)ell * n) : nullptr);
                    sfp_automorph(s->dev, i ? cb.back()->ptr : out->c0, x->c0, gal, st->qmap(ell));
                    sfp_automorph(s->dev, tb.back()->ptr, x->c1, gal, st->qmap(ell));
                    sfp_modup_inner_phase(s->dev, nullptr, nullptr, tb.back()->ptr, ell, K, s->Lq, s->alpha,
                                          convs.data(), nullptr, nullptr, nullptr, 0, 0, ~0u, eb.back()->ptr,
                                          sb.back()->ptr, 1);
                }
            }
            for (size_t i = b0; i < b1; ++i) {
                const size_t k = i - b0;
                if (i && oneSum) c0s.push_back(cb[k]);
                else if (i) sfp_add(s->dev, out->c0, out->c0, cb[k]->ptr, st->qmap(ell));
                sfp_modup_inner_phase(s->dev, acc->ptr, acc->ptr + stride, tb[k]->ptr, ell, K, s->Lq, s->alpha,
                                      convs.data(), (*keys[i])->ptr, nullptr, nullptr, 0, i ? 1 : 0,
                                      i + 1 == rot.size() ? ell : ~0u, eb[k]->ptr, sb[k]->ptr, 2);
                s->stats.automorph++;
                s->stats.keyswitch++;
                s->countBytes((5.0 * ell + 2.0 * beta * (ell + K)) * n * 8);
            }
        }
        if (!c0s.empty()) {
            std::vector<const uint64_t*> ins{out->c0};
            for (auto& b : c0s) ins.push_back(b->ptr);
            const std::vector<uint64_t> ones(ins.size() * ell, 1);
            sfp_lin_wsum(s->dev, out->c0, ins.data(), ones.data(), (uint32_t)ins.size(), st->qmap(ell));
        }
        rowDone = 1;
    }
    auto t = rowDone ? nullptr : s->alloc((size_t)s->rows(ell) * n);
    auto c0 = rowDone ? nullptr : s->alloc((size_t)s->rows(ell) * n);
    auto ext = shard ? s->alloc(stride * beta) : nullptr;  // (the unsharded ModUp allocates its own)
    for (size_t i = 0; i < (rowDone ? 0 : rot.size()); ++i) {
        const Ciphertext<DCRTPoly>& x = a[rot[i]];
        const uint32_t gal = GaloisForRotation(r[rot[i]]);
        // c0' = sum sigma_k(c0_k) (+ the shared ModDown below)
        sfp_automorph(s->dev, i ? c0->ptr : out->c0, x->c0, gal, st->qmap(ell));
        if (i) sfp_add(s->dev, out->c0, out->c0, c0->ptr, st->qmap(ell));
        sfp_automorph(s->dev, t->ptr, x->c1, gal, st->qmap(ell));
        if (shard) {
            SfheInternal::modupShard(s, ext->ptr, t->ptr, ell);
            SfheInternal::innerShard(s, acc->ptr, ext->ptr, stride, beta, ell, *keys[i], i ? 1 : 0);
        } else {
            // the last term's pass also runs the ModDown's first inverse pass on the P rows
            rowDone = SfheInternal::modupInner(this, acc->ptr, t->ptr, ell, *keys[i], nullptr, nullptr, 0, i ? 1 : 0,
                                               i + 1 == rot.size() ? ell : ~0u);
        }
        s->stats.automorph++;
        s->stats.keyswitch++;
        s->countBytes((5.0 * ell + 2.0 * beta * (ell + K)) * n * 8);
    }
    if (shard) {
        SfheInternal::modDownShard(s, acc->ptr, ell, out->c0, out->c1, 1, 0);
    } else {
        auto md = s->alloc((size_t)2 * ell * n);
        sfp_moddown2(s->dev, out->c0, out->c1, acc->ptr, stride, ell, K, s->Lq, s->moddownConvOf(tier),
                     s->pInvModQof(tier), 1, 0, md->ptr, rowDone);
    }
    Ciphertext<DCRTPoly> res = SfheInternal::traced(this, out, "EvalRotateSum");
    for (size_t k : ident) res = EvalAdd(res, a[k]);
    return res;
}

// Double hoisting (Bossuat et al.'s hoisted ModDown): with acc_k the
// extended-basis inner product of rotation k, p (.) ModDown(acc_k) and
// ModDown(p_ext (.) acc_k) are the same value up to the ModDown rounding, so
// sum_k p_k (.) Rot_k(a) = sum_k p_k (.) sigma_k(c0) + ModDown(sum_k p_k,ext (.) acc_k)
// takes one ModDown for the whole sum; the diagonal's rounding is also no
// longer multiplied by p_k.  Unsharded contexts (bootstrapping's linear maps).
Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalRotMultAddHoisted(
    const std::vector<Ciphertext<DCRTPoly>>& a,
    const std::vector<std::vector<std::pair<int32_t, Plaintext>>>& terms) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (a.empty() || a.size() != terms.size()) SFHE_THROW("EvalRotMultAddHoisted: operand count mismatch");
    if (s->sharded) SFHE_THROW("EvalRotMultAddHoisted: sharded contexts are not supported");
    SfheInternal::depsv(s, a);
    const uint32_t level = a[0]->level;
    uint32_t slots = 0;
    for (size_t t = 0; t < a.size(); ++t) {
        if (a[t]->level != level) SFHE_THROW("EvalRotMultAddHoisted: inputs at different levels");
        slots = std::max(slots, a[t]->slots);
        for (const auto& tk : terms[t]) slots = std::max(slots, tk.second->slots);
    }
    const uint32_t ell = s->ellOf(level), n = s->n, K = s->K;
    if (ell < 2) SFHE_THROW("no levels left (multiplicative depth exhausted)");
    const uint32_t beta = (ell + s->alpha - 1) / s->alpha;
    const size_t stride = (size_t)(ell + K) * n, pw = s->polyWords(level);
    const sfp_limbs q = s->qmap(ell);
    auto prod = s->alloc(2 * pw);  // the product sum before its rescale
    uint64_t* t0 = prod->ptr;
    uint64_t* t1 = t0 + pw;
    auto acc = s->alloc(2 * stride);
    bool accOn = false;
    std::vector<DeviceBufferPtr> keep;
    std::vector<const uint64_t*> x0, m0, x1, m1;  // c0 terms; c1 terms of the unrotated diagonals
    for (size_t t = 0; t < a.size(); ++t) {
        DeviceBufferPtr ext;
        for (const auto& [r, pt] : terms[t]) {
            const uint64_t* m = SfheInternal::encoded(this, pt, level);
            const uint32_t gal = GaloisForRotation(r);
            if (gal == 1) {
                x0.push_back(a[t]->c0);
                m0.push_back(m);
                x1.push_back(a[t]->c1);
                m1.push_back(m);
                continue;
            }
            auto it = s->rotKeys.find(gal);
            if (it == s->rotKeys.end())
                SFHE_THROW("EvalKey for rotation " + std::to_string(r) + " is not found");
            if (!ext) {  // the input's ModUp, shared by its rotations
                ext = s->alloc(stride * beta);
                auto scratch = s->alloc((size_t)ell * n);
                sfp_modup(s->dev, ext->ptr, a[t]->c1, ell, K, s->Lq, s->alpha,
                          SfheInternal::modupConv(this, ell).data(), scratch->ptr);
            }
            auto rc0 = s->alloc(pw);
            sfp_automorph(s->dev, rc0->ptr, a[t]->c0, gal, q);
            x0.push_back(rc0->ptr);
            m0.push_back(m);
            keep.push_back(rc0);
            // the shared digits read through sigma by the inner product (as
            // EvalFastRotation; SFHE_KS_AUT=0: a permuted copy per rotation)
            static const bool autFused = [] {
                const char* v = std::getenv("SFHE_KS_AUT");
                return !v || *v != '0';
            }();
            if (autFused) {
                sfp_ks_inner_mul_aut(s->dev, acc->ptr, acc->ptr + stride, ext->ptr, stride, it->second->ptr, beta, ell,
                                     K, s->Lq, SfheInternal::encodedExt(this, pt, level), accOn ? 1 : 0, gal);
            } else {
                auto rext = s->alloc(stride * beta);
                const uint32_t rows = beta * (ell + K);
                sfp_automorph(s->dev, rext->ptr, ext->ptr, gal, sfp_limbs{rows, rows, 0, 0});
                sfp_ks_inner_mul(s->dev, acc->ptr, acc->ptr + stride, rext->ptr, stride, it->second->ptr, beta, ell,
                                 K, s->Lq, SfheInternal::encodedExt(this, pt, level), accOn ? 1 : 0);
            }
            accOn = true;
            s->stats.keyswitch++;
            s->stats.automorph++;
            s->countBytes((3.0 * ell + (2.0 * beta + 5.0) * (ell + K)) * n * 8);
        }
    }
    auto macInto = [&](uint64_t* out, const std::vector<const uint64_t*>& x, const std::vector<const uint64_t*>& m) {
        if (x.empty()) {
            sfp_zero(s->dev, out, pw * 8);
            return;
        }
        for (size_t done = 0; done < x.size(); done += SFP_MAX_WSUM) {
            const uint32_t take = (uint32_t)std::min<size_t>(SFP_MAX_WSUM, x.size() - done);
            if (done == 0) {
                sfp_mac_plain(s->dev, out, x.data(), m.data(), take, q);
            } else {
                auto part = s->alloc(pw);
                sfp_mac_plain(s->dev, part->ptr, x.data() + done, m.data() + done, take, q);
                sfp_add(s->dev, out, out, part->ptr, q);
            }
        }
    };
    macInto(t0, x0, m0);
    macInto(t1, x1, m1);
    s->stats.ptmult += x0.size() + x1.size();
    s->countBytes((2.0 * x0.size() + 2.0 * x1.size() + 2.0) * ell * n * 8);
    if (accOn) {
        auto scratch = s->alloc((size_t)2 * ell * n);
        sfp_moddown2(s->dev, t0, t1, acc->ptr, stride, ell, K, s->Lq, s->moddownConv, s->pInvModQ.data(), 1, 1,
                     scratch->ptr, 0);
    }
    return SfheInternal::traced(this, SfheInternal::rescale(this, t0, t1, level, slots), "EvalRotMultAddHoisted");
}

// ============================================================================
// fused weighted sum (Chebyshev leaves, EvalPolyLinear)

// sum_j w_j * (c0_j, c1_j) at `level` (canonical scale), then one rescale
namespace {
// residue of round(w * Delta_level^2 / inScale) modulo each of the ell primes:
// the weight of a ciphertext of scale inScale (Delta_level unless an input of
// a lower level enters unadjusted) whose product, at scale Delta_level^2, is
// rescaled to the next level
void weightResidues(const SfheContextState* s, double w, uint32_t level, uint32_t ell,
                    std::vector<uint64_t>& kk, double inScale = 0.0) {
    const double K = inScale > 0.0 ? w * s->scale[level] * (s->scale[level] / inScale) : w * s->scale[level];
    const double r = std::nearbyint(K);
    const bool neg = r < 0;
    const double a = std::fabs(r);
    u128 v;
    if (a < 1.8e19) {
        v = (u128)(u64)a;
    } else {
        const double hi = std::floor(std::ldexp(a, -64));
        v = ((u128)(u64)hi << 64) + (u128)(u64)(a - std::ldexp(hi, 64));
    }
    for (uint32_t i = 0; i < s->rows(ell); ++i) {  // the local rows' primes
        const u64 q = s->primes[s->qprime(i, ell)];
        const u64 m = (u64)(v % q);
        kk.push_back(neg ? (m ? q - m : 0) : m);
    }
}
}  // namespace

std::vector<Ciphertext<DCRTPoly>> CryptoContextImpl<DCRTPoly>::LinearWSumRescaleMulti(
    const std::vector<const uint64_t*>& in0, const std::vector<const uint64_t*>& in1,
    const std::vector<std::vector<double>>& w, uint32_t level, uint32_t slots, const std::vector<double>* inScale) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    const uint32_t ell = s->ellOf(level), n = s->n;
    const uint32_t nin = (uint32_t)in0.size(), nout = (uint32_t)w.size();
    if (ell < 2) SFHE_THROW("no levels left (multiplicative depth exhausted)");
    if (nin == 0 || nin > SFP_MAX_WSUM || nout == 0) SFHE_THROW("LinearWSumRescaleMulti: bad sizes");
    if (inScale && inScale->size() != nin) SFHE_THROW("LinearWSumRescaleMulti: scale count");
    std::vector<uint64_t> kk;
    kk.reserve((size_t)nout * nin * s->rows(ell));
    for (const auto& row : w) {
        if (row.size() != nin) SFHE_THROW("LinearWSumRescaleMulti: weight row size");
        for (uint32_t j = 0; j < nin; ++j) weightResidues(s, row[j], level, ell, kk, inScale ? (*inScale)[j] : 0.0);
    }
    const size_t pw = s->polyWords(level);  // words per polynomial
    auto sums = s->alloc((size_t)nout * 2 * pw);
    sfp_lin_wsum_multi(s->dev, sums->ptr, 2 * pw, pw, in0.data(), in1.data(), nin, kk.data(), nout,
                       s->qmap(ell));
    // one rescale of all 2 * nout polynomials; the results share one buffer
    const size_t qw = s->polyWords(level + 1);
    auto res = s->alloc((size_t)nout * 2 * qw);
    if (s->shardAt(ell))
        SfheInternal::rescaleShard(s, res->ptr, sums->ptr, ell, 2 * nout, pw, qw);
    else
        sfp_rescale(s->dev, res->ptr, sums->ptr, ell, s->qInvTable[ell].data(), 2 * nout, pw, qw);
    std::vector<Ciphertext<DCRTPoly>> out(nout);
    for (uint32_t o = 0; o < nout; ++o) {
        auto ct = std::make_shared<CiphertextImpl<DCRTPoly>>();
        ct->cc = shared_from_this();
        ct->buf = res;
        ct->c0 = res->ptr + (size_t)o * 2 * qw;
        ct->c1 = ct->c0 + qw;
        ct->level = level + 1;
        ct->slots = slots;
        ct->scale = s->scale[level + 1];
        out[o] = ct;
    }
    s->stats.wsum_terms += (uint64_t)nin * nout;
    s->stats.rescale += 2 * nout;
    s->countBytes(((double)nin + nout) * 2.0 * pw * 8 + 4.0 * pw * 8 * nout);
    return out;
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::LinearWSumRescale(
    const std::vector<const uint64_t*>& in0, const std::vector<const uint64_t*>& in1,
    const std::vector<double>& w, uint32_t level, uint32_t slots, const std::vector<double>* inScale) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    const uint32_t ell = s->ellOf(level);
    if (ell < 2) SFHE_THROW("no levels left (multiplicative depth exhausted)");
    if (inScale && inScale->size() != w.size()) SFHE_THROW("LinearWSumRescale: scale count");
    const size_t pw = s->polyWords(level);
    auto tmp = s->alloc(2 * pw);
    uint64_t* t0 = tmp->ptr;
    uint64_t* t1 = t0 + pw;
    const sfp_limbs q = s->qmap(ell);
    // chunks of SFP_MAX_WSUM terms accumulate through the extra "previous sum" input
    size_t done = 0;
    bool first = true;
    while (done < w.size()) {
        size_t take = std::min<size_t>(w.size() - done, SFP_MAX_WSUM - (first ? 0 : 1));
        std::vector<const uint64_t*> a0, a1;
        std::vector<uint64_t> kk;
        if (!first) {
            a0.push_back(t0);
            a1.push_back(t1);
            for (uint32_t i = 0; i < s->rows(ell); ++i) kk.push_back(1);
        }
        for (size_t j = done; j < done + take; ++j) {
            a0.push_back(in0[j]);
            a1.push_back(in1[j]);
            // product scale Delta_l^2 -> rescale -> Delta_{l+1}
            weightResidues(s, w[j], level, ell, kk, inScale ? (*inScale)[j] : 0.0);
        }
        sfp_lin_wsum(s->dev, t0, a0.data(), kk.data(), (uint32_t)a0.size(), q);
        sfp_lin_wsum(s->dev, t1, a1.data(), kk.data(), (uint32_t)a1.size(), q);
        s->stats.wsum_terms += take;
        s->countBytes((double)(a0.size() + 1) * 2.0 * ell * s->n * 8);
        done += take;
        first = false;
    }
    return SfheInternal::traced(this, SfheInternal::rescale(this, t0, t1, level, slots), "LinearWSumRescale");
}


// ============================================================================
// level management

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::Rescale(const Ciphertext<DCRTPoly>& a) {
    Settle(a);  // a lazy product's pending rescale
    return a->Clone();
}

void CryptoContextImpl<DCRTPoly>::Settle(const Ciphertext<DCRTPoly>& ct) {
    if (!ct) return;
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&ct});
}

void CryptoContextImpl<DCRTPoly>::LevelReduceInPlace(Ciphertext<DCRTPoly>& a, std::nullptr_t,
                                                     size_t levels) {
    a = AdjustLevel(a, a->level + (uint32_t)levels);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::AdjustLevel(const Ciphertext<DCRTPoly>& a,
                                                             uint32_t targetLevel) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    auto r = SfheInternal::adjust(this, a, targetLevel);
    return r == a ? a->Clone() : r;
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::AdjustLevelScaled(const Ciphertext<DCRTPoly>& a,
                                                                   uint32_t targetLevel, double factor) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    auto r = SfheInternal::adjust(this, a, targetLevel, factor);
    return r == a ? a->Clone() : r;
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::ModRaise(const Ciphertext<DCRTPoly>& a) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    SfheContextState* s = st.get();
    if (s->sharded) SFHE_THROW("bootstrapping a limb-sharded context is not supported");
    if (s->ellOf(a->level) != 1) SFHE_THROW("ModRaise needs a ciphertext at the last level (one limb)");
    const uint32_t n = s->n;
    // coefficient form of both single-limb polys, then their centred lift to
    // every Q limb, NTT'd there -- on the device: the rescale-with-given-row
    // prim computes (in - [last]_{q_i}) * k_i; with in = 0 and k_i = -1 that is
    // [last]_{q_i} (no host round trip, so bootstrapping can be captured)
    auto t = s->alloc(2 * (size_t)n);
    sfp_d2d(s->dev, t->ptr, a->c0, (size_t)n * 8);
    sfp_d2d(s->dev, t->ptr + n, a->c1, (size_t)n * 8);
    sfp_ntt(s->dev, t->ptr, sfp_limbs{1, 1, 0, 0, 0}, 1);
    sfp_ntt(s->dev, t->ptr + n, sfp_limbs{1, 1, 0, 0, 0}, 1);
    auto out = SfheInternal::newCt(this, 0, a->slots);
    const size_t pw = s->polyWords(0);
    auto zero = s->alloc(2 * pw);
    sfp_zero(s->dev, zero->ptr, 2 * pw * 8);
    std::vector<uint64_t> minus1(s->Lq);
    for (uint32_t i = 0; i < s->Lq; ++i) minus1[i] = s->primes[i] - 1;
    sfp_rescale_rows(s->dev, out->c0, zero->ptr, t->ptr, 0, s->qmap(s->Lq), minus1.data(), 2, pw,
                     (size_t)(out->c1 - out->c0), n);
    s->wrote(out->buf.get());
    return SfheInternal::traced(this, out, "ModRaise");
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalConjugate(const Ciphertext<DCRTPoly>& a) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&a});
    SfheContextState* s = st.get();
    const uint32_t gal = 2 * s->n - 1;  // X -> X^-1: complex conjugation of every slot
    auto it = s->rotKeys.find(gal);
    if (it == s->rotKeys.end()) SFHE_THROW("conjugation key not found (EvalConjugateKeyGen)");
    const uint32_t ell = s->ellOf(a->level);
    auto out = SfheInternal::newCt(this, a->level, a->slots);
    auto t = s->alloc(s->polyWords(a->level));
    sfp_automorph(s->dev, out->c0, a->c0, gal, st->qmap(ell));
    sfp_automorph(s->dev, t->ptr, a->c1, gal, st->qmap(ell));
    s->stats.automorph++;
    SfheInternal::keySwitch(this, t->ptr, ell, it->second, out->c0, out->c1, 1, 0);
    return SfheInternal::traced(this, out, "EvalConjugate");
}

void CryptoContextImpl<DCRTPoly>::EvalConjugateKeyGen(const PrivateKey<DCRTPoly>& sk) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    const uint32_t gal = 2 * s->n - 1;
    if (s->rotKeys.count(gal)) return;
    const uint32_t NP = s->Lq + s->K;
    auto sg = s->alloc((size_t)NP * s->n);
    sfp_automorph(s->dev, sg->ptr, sk->s->ptr, gal, sfp_limbs{NP, NP, 0});
    s->rotKeys[gal] = SfheInternal::genSwitchKey(this, sg->ptr, sk->s->ptr);
    SfheInternal::genTierKeys(this, sg->ptr, sk->s->ptr, gal);
}

// ============================================================================
// limb sharding

void CryptoContextImpl<DCRTPoly>::EnableSharding(int rank, int world, bool shardAtOne) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (world < 1 || rank < 0 || rank >= world) SFHE_THROW("EnableSharding: bad rank / world");
    if (s->relinKey || !s->rotKeys.empty()) SFHE_THROW("EnableSharding must precede the key generation");
    if (s->sharded) SFHE_THROW("EnableSharding: already sharded");
    s->rank = rank;
    s->world = world;
    s->ptCache.clear();
    s->ptCacheBytes = 0;
    if (world == 1 && !shardAtOne) return;
    s->sharded = true;
    // replicated tail: levels of at most SFHE_SHARD_TAIL Q limbs (default 16)
    // run on every rank without exchanges
    const char* t = std::getenv("SFHE_SHARD_TAIL");
    s->tailLimbs = t && *t ? (uint32_t)std::atoi(t) : 16u;
    // P -> this rank's Q rows (targets in local row order; a level's rows are a prefix)
    std::vector<uint32_t> src, dst;
    for (uint32_t k = 0; k < s->K; ++k) src.push_back(s->Lq + k);
    for (uint32_t i = 0; i < s->owned(s->Lq); ++i) dst.push_back(s->qprimeShard(i));
    s->moddownConvShard = dst.empty() ? nullptr : SfheInternal::makeConv(s, src, dst);
    // Sliced keys (each GPU stores only its slice of every
    // evaluation key): rows of the replicated levels, of this rank's dealt
    // primes and the P rows.  SFHE_KEY_SLICE=0 keeps whole keys.
    const char* ks = std::getenv("SFHE_KEY_SLICE");
    if (world > 1 && !(ks && *ks == '0')) {
        sfp_key_geom& g = s->kgeom;
        g.tail = std::min(s->tailLimbs, s->Lq);
        g.world = (uint32_t)world;
        g.lq = s->Lq;
        g.first = g.tail + ((uint32_t)rank + world - g.tail % world) % world;
        uint32_t high = 0;
        for (uint32_t p = g.first; p < s->Lq; p += world) ++high;
        g.pstart = g.tail + high;
        g.rows = g.pstart + s->K;
        sfp_set_key_geom(s->dev, &g);
    }
}

uint32_t CryptoContextImpl<DCRTPoly>::ShardTailLimbs() const { return st->sharded ? st->tailLimbs : 0; }
uint32_t CryptoContextImpl<DCRTPoly>::SwitchKeyRows() const { return st->keyRows(); }

void CryptoContextImpl<DCRTPoly>::EnableBatchGroups(int group, int groups, bool gatherAtOne) {
    OpLock g(st.get());
    if (groups < 1 || group < 0 || group >= groups) SFHE_THROW("EnableBatchGroups: bad group / groups");
    if (st->capturing) SFHE_THROW("EnableBatchGroups inside a capture");
    st->bgroup = group;
    st->bgroups = groups;
    st->bgatherAtOne = gatherAtOne;
}
bool CryptoContextImpl<DCRTPoly>::BatchGather() const { return st->bgroups > 1 || st->bgatherAtOne; }
int CryptoContextImpl<DCRTPoly>::BatchGroup() const { return st->bgroup; }
int CryptoContextImpl<DCRTPoly>::BatchGroups() const { return st->bgroups; }

std::vector<Ciphertext<DCRTPoly>> CryptoContextImpl<DCRTPoly>::GatherGroups(const Ciphertext<DCRTPoly>& ct) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (!ct) SFHE_THROW("GatherGroups: null ciphertext");
    SfheInternal::deps(s, {&ct});
    const size_t pw = s->polyWords(ct->level);
    const size_t G = (size_t)s->bgroups;
    // [c0 rows][c1 rows] of this group, then every group's, group-major
    auto recv = s->alloc(G * 2 * pw);
    uint64_t* mine = recv->ptr + (size_t)s->bgroup * 2 * pw;
    sfp_d2d(s->dev, mine, ct->c0, pw * 8);
    sfp_d2d(s->dev, mine + pw, ct->c1, pw * 8);
    sfp_group_allgather(s->dev, mine, recv->ptr, 2 * pw * 8);
    std::vector<Ciphertext<DCRTPoly>> out(G);
    for (size_t i = 0; i < G; ++i) {
        auto c = std::make_shared<CiphertextImpl<DCRTPoly>>(*ct);
        c->buf = recv;
        c->c0 = recv->ptr + i * 2 * pw;
        c->c1 = c->c0 + pw;
        c->def.reset();
        c->pend = false;
        c->undo.reset();
        out[i] = c;
    }
    return out;
}

int CryptoContextImpl<DCRTPoly>::ShardRank() const { return st->rank; }
int CryptoContextImpl<DCRTPoly>::ShardWorld() const { return st->world; }
bool CryptoContextImpl<DCRTPoly>::IsSharded() const { return st->sharded; }

void CryptoContextImpl<DCRTPoly>::RowsAt(const Ciphertext<DCRTPoly>& ct, uint32_t level, const uint64_t** c0,
                                         const uint64_t** c1, std::vector<DeviceBufferPtr>& keep) {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    SfheInternal::deps(s, {&ct});
    const uint32_t ell = s->ellOf(level);
    if (level < ct->level) SFHE_THROW("RowsAt: a ciphertext's rows cannot be read at a higher limb count");
    if (s->shardAt(s->ellOf(ct->level)) && !s->shardAt(ell)) {
        auto full = SfheInternal::gatherRows(s, ct->c0, ct->c1, ell);
        *c0 = full->ptr;
        *c1 = full->ptr + (size_t)ell * s->n;
        keep.push_back(std::move(full));
        return;
    }
    *c0 = ct->c0;
    *c1 = ct->c1;
}

void CryptoContextImpl<DCRTPoly>::DownloadRows(const Ciphertext<DCRTPoly>& ct, uint64_t* out) {
    OpLock g(st.get());
    SfheInternal::deps(st.get(), {&ct});
    SfheContextState* s = st.get();
    const size_t words = (size_t)s->ellOf(ct->level) * s->n;
    if (s->sharded) {  // collective: every rank receives every row
        auto full = SfheInternal::gatherFull(s, ct);
        sfp_d2h(s->dev, out, full->ptr, 2 * words * 8);
    } else {
        sfp_d2h(s->dev, out, ct->c0, words * 8);
        sfp_d2h(s->dev, out + words, ct->c1, words * 8);
    }
    const char* e = sfp_last_error(s->dev);
    if (e) SFHE_THROW(std::string("device error: ") + e);
}

// ============================================================================
// graph capture (engine extension)

struct CryptoContextImpl<DCRTPoly>::CapturedGraph {
    std::weak_ptr<CryptoContextImpl<DCRTPoly>> cc;
    sfp_graph* g = nullptr;
    std::vector<std::pair<uint64_t*, size_t>> owned;  // pool blocks the graph addresses
    Ciphertext<DCRTPoly> keep;
    ~CapturedGraph() {
        keep.reset();
        auto c = cc.lock();
        if (!c) return;  // the context is gone (or releasing it: ReleaseGraph ran)
        c->ReleaseGraph(*this);
    }
};

void CryptoContextImpl<DCRTPoly>::ReleaseGraph(CapturedGraph& cg) {
    SfheContextState* s = st.get();
    OpLock lk(s);
    cg.keep.reset();
    if (cg.g) sfp_graph_destroy(s->dev, cg.g);  // drains the device first
    cg.g = nullptr;
    std::lock_guard<std::mutex> pg(s->poolMu);
    for (auto& o : cg.owned) {
        auto it = s->graphOwned.find(o.first);
        if (it == s->graphOwned.end()) continue;
        const bool live = it->second;
        s->graphOwned.erase(it);
        if (!live) s->freeList[0][o.second].push_back(o.first);  // else its holder frees it
    }
    cg.owned.clear();
    cg.cc.reset();
}

bool CryptoContextImpl<DCRTPoly>::BeginCapture() {
    OpLock g(st.get());
    SfheContextState* s = st.get();
    if (s->capturing) SFHE_THROW("BeginCapture: a capture is already open");
    if (s->forkedLanes) SFHE_THROW("BeginCapture inside a lane region");
    // a host transport synchronises (no capture); RCCL collectives are captured
    if ((s->sharded || s->bgroups > 1 || s->bgatherAtOne) && !sfp_comm_capturable(s->dev)) return false;
    sfp_sync(s->dev);
    if (sfp_capture_begin(s->dev) != 0) {
        std::fprintf(stderr, "sfhe: this backend cannot capture graphs (%s); sorting eagerly\n", sfp_backend_name());
        return false;
    }
    s->capturing = true;
    s->captureEpoch = ++s->epochCount;
    s->capAllocs.clear();
    // every cross-lane dependency inside the region must become a graph edge
    std::memset(s->synced, 0, sizeof s->synced);
    return true;
}

std::shared_ptr<CryptoContextImpl<DCRTPoly>::CapturedGraph> CryptoContextImpl<DCRTPoly>::EndCapture(
    const Ciphertext<DCRTPoly>& keep) {
    OpLock lk(st.get());
    SfheContextState* s = st.get();
    if (!s->capturing) SFHE_THROW("EndCapture without BeginCapture");
    // the graph must write the kept result's final rows: a lazy result is
    // settled inside the region
    if (keep) SfheInternal::deps(s, {&keep});
    sfp_graph* g = sfp_capture_end(s->dev);
    s->capturing = false;
    if (!g) s->abandonedEpochs.insert(s->captureEpoch);  // its encodings are stale (encoded())
    s->captureEpoch = 0;
    std::memset(s->synced, 0, sizeof s->synced);
    std::vector<std::pair<uint64_t*, size_t>> blocks;
    {
        std::lock_guard<std::mutex> pg(s->poolMu);
        blocks.swap(s->capAllocs);
    }
    if (!g) {
        const char* e = sfp_last_error(s->dev);
        std::fprintf(stderr, "sfhe: graph capture abandoned, running eagerly (%s)\n", e ? e : "unknown");
        sfp_clear_error(s->dev);  // not a device fault: the eager rerun must not inherit it
        return nullptr;
    }
    auto out = std::make_shared<CapturedGraph>();
    out->cc = shared_from_this();
    out->g = g;
    out->keep = keep;
    std::sort(blocks.begin(), blocks.end());
    blocks.erase(std::unique(blocks.begin(), blocks.end()), blocks.end());
    std::lock_guard<std::mutex> pg(s->poolMu);
    // a recorded block is either back in a free list (the region freed it:
    // take it out, the graph owns it now) or still held (the result, keep)
    std::unordered_map<uint64_t*, size_t> want(blocks.begin(), blocks.end());
    auto scrub = [&](std::map<size_t, std::vector<uint64_t*>>& fl) {
        for (auto& kv : fl) {
            auto& v = kv.second;
            v.erase(std::remove_if(v.begin(), v.end(),
                                   [&](uint64_t* p) {
                                       auto it = want.find(p);
                                       if (it == want.end()) return false;
                                       s->graphOwned[p] = false;
                                       return true;
                                   }),
                    v.end());
        }
    };
    for (auto& fl : s->freeList) scrub(fl);
    scrub(s->forkPool);
    for (auto& b : blocks)
        if (!s->graphOwned.count(b.first)) s->graphOwned[b.first] = true;  // live
    out->owned = std::move(blocks);
    return out;
}

void CryptoContextImpl<DCRTPoly>::Launch(const std::shared_ptr<CapturedGraph>& g) {
    OpLock lk(st.get());
    SfheContextState* s = st.get();
    if (!g || !g->g) SFHE_THROW("Launch: no graph");
    if (s->forkedLanes) SFHE_THROW("Launch inside a lane region");
    sfp_graph_launch(s->dev, g->g);
    // the graph ran (stream-ordered) on lane 0: so did every write it made
    if (g->keep) s->wrote(g->keep->buf.get());
}

bool CryptoContextImpl<DCRTPoly>::GraphFamilyTime(const std::shared_ptr<CapturedGraph>& g, uint32_t family,
                                                  int reps, double* ms, uint64_t* launches, double* bytes) {
    if (!g || !g->g) return false;
    OpLock lk(st.get());
    return sfp_graph_family_time(st->dev, g->g, family, reps, ms, launches, bytes) == 0;
}

size_t CryptoContextImpl<DCRTPoly>::GraphNodes(const std::shared_ptr<CapturedGraph>& g) const {
    return g ? sfp_graph_nodes(g->g) : 0;
}

void CryptoContextImpl<DCRTPoly>::CopyCiphertextInto(const Ciphertext<DCRTPoly>& dst,
                                                     const Ciphertext<DCRTPoly>& src) {
    OpLock lk(st.get());
    SfheContextState* s = st.get();
    // the destination's rows are what a graph reads: settling a lazy one would
    // move it to a new buffer the graph never sees
    if (dst->def || dst->pend || dst->undo) SFHE_THROW("CopyCiphertextInto: the destination is a lazy product");
    SfheInternal::deps(s, {&dst, &src});
    if (dst->level != src->level) SFHE_THROW("CopyCiphertextInto: level mismatch");
    const size_t bytes = s->polyWords(src->level) * 8;
    sfp_d2d(s->dev, dst->c0, src->c0, bytes);
    sfp_d2d(s->dev, dst->c1, src->c1, bytes);
    s->wrote(dst->buf.get());
}

// ============================================================================
// bootstrapping: the k-way / bitonic rows are next;
// link-compatible entry points throw until then.

}  // namespace lbcrypto
