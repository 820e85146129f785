// Internal state of a CKKS context (not part of the public API).
#pragma once
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "modarith.h"
#include "openfhe.h"

namespace lbcrypto {

class DeviceBuffer {
  public:
    DeviceBuffer(SfheContextState* s, uint64_t* p, size_t w, int l, uint64_t r)
        : st(s), ptr(p), words(w), lane(l), region(r) {}
    ~DeviceBuffer();
    SfheContextState* st;
    uint64_t* ptr;
    size_t words;
    int lane;                      // lane of the last writer (allocating lane until an in-place write)
    uint64_t region;               // fork/join region it was allocated in (0: none)
    uint64_t seq = 0;              // position of its last write in lane's sequence
    int ksTier = -1;               // a switching key: its special-prime tier (-1: the whole P)
    sfp_event* ready = nullptr;    // shared encodings: end of the producing work
    uint64_t readyEpoch = 0;       // capture epoch `ready` was recorded in (0: none)
    uint64_t capEpoch = 0;         // capture epoch it was allocated in (0: none)
    std::shared_ptr<DeviceBuffer> parent;  // a view into parent's block (batched encodings)
};

struct BootstrapPrecomp;  // bootstrap.cpp

// A product whose rescale is deferred to its first consumer (lazy
// rescaling, context.cpp): run() fills ct's rows either in the canonical
// form (the fused product + rescale) or, pending = true, before the rescale.
struct DeferredOp {
    virtual ~DeferredOp() = default;
    virtual void run(CryptoContextImpl<DCRTPoly>* cc, CiphertextImpl<DCRTPoly>& ct, bool pending) = 0;
};

struct PtCacheEntry {
    std::vector<std::complex<double>> values;
    uint32_t slots;
    DeviceBufferPtr buf;
};

// A special-prime tier: key switches at ell <= maxEll limbs
// (a single digit, beta = 1) run over the first K special primes P' only,
// P' >= Q_maxEll * 2^20 as the context's P >= its largest digit * 2^20 --
// the same noise margin with fewer extended rows (the metric context, K = 13:
// K' = 3 / 5 / 7 / 9 / 11 up to 2 / 4 / 6 / 8 / 10 limbs).  Its keys are
// another set (one digit, b rows then a rows over the Q primes and P'),
// generated with the context's keys.
struct KsTier {
    uint32_t maxEll = 0, K = 0;
    std::vector<uint64_t> pModQ, pInvModQ;  // P' mod q_i, P'^-1 mod q_i
    sfp_conv* moddownConv = nullptr;        // P' -> Q
    std::map<uint32_t, std::vector<sfp_conv*>> modupConv;  // ell -> Q_ell -> P'
    DeviceBufferPtr relinKey;
    std::map<uint32_t, DeviceBufferPtr> rotKeys;
};

struct SfheContextState {
    CCParams<CryptoContextCKKSRNS> params;
    uint32_t n = 0, logn = 0;
    uint32_t L = 0;   // multiplicative depth
    uint32_t Lq = 0;  // number of Q primes = L+1
    uint32_t K = 0;   // number of P primes
    uint32_t dnum = 0, alpha = 0;
    uint32_t batch = 0;
    std::vector<uint64_t> primes;  // [q_0..q_L, p_0..p_{K-1}] (+ q_ext when ext)
    // FLEXIBLEAUTOEXT: fresh encryptions are formed modulo Q*q_ext and
    // rescaled by q_ext, so their noise is divided away (extIdx = Lq+K)
    bool ext = false;
    uint32_t extIdx = 0;
    std::vector<uint64_t> extInvModQ;  // q_ext^{-1} mod q_i
    std::vector<uint64_t> extModQ;     // q_ext mod q_i
    std::vector<sf_barrett> bar;
    std::vector<double> scale;  // canonical scale of each level 0..L
    sfp_dev* dev = nullptr;

    // base-conversion tables
    std::map<uint32_t, std::vector<sfp_conv*>> modupConv;  // ell -> per digit
    sfp_conv* moddownConv = nullptr;                        // P -> Q (all Lq targets)
    std::vector<uint64_t> pInvModQ;                         // P^{-1} mod q_i
    std::vector<uint64_t> pModQ;                            // P mod q_i
    std::vector<std::vector<uint64_t>> qInvTable;  // [ell][i] = q_{ell-1}^{-1} mod q_i
    uint32_t tablePrimes() const { return Lq + K + (ext ? 1 : 0); }

    // keys (of the key pair tagged keyTag; 0 until a key generation or a
    // deserialized key record claims the context)
    uint64_t keyTag = 0;
    DeviceBufferPtr relinKey;
    std::map<uint32_t, DeviceBufferPtr> rotKeys;  // galois -> key
    std::set<int32_t> rotIndices;
    // special-prime tiers, ascending maxEll (SFHE_KS_TIERS; replicated levels only when sharded)
    std::vector<KsTier> tiers;
    bool tiersReady = true;  // false once keys arrive without their tier keys (deserialized)
    // the tier of a key switch at ell limbs (-1: the whole P)
    int tierAt(uint32_t ell) const {
        if (!tiersReady || shardAt(ell)) return -1;  // (dealt levels: the exchanges use the whole P)
        for (size_t t = 0; t < tiers.size(); ++t)
            if (ell <= tiers[t].maxEll) return (int)t;
        return -1;
    }
    uint32_t Kof(int t) const { return t < 0 ? K : tiers[(size_t)t].K; }
    const uint64_t* pModQof(int t) const { return t < 0 ? pModQ.data() : tiers[(size_t)t].pModQ.data(); }
    const uint64_t* pInvModQof(int t) const { return t < 0 ? pInvModQ.data() : tiers[(size_t)t].pInvModQ.data(); }
    sfp_conv* moddownConvOf(int t) const { return t < 0 ? moddownConv : tiers[(size_t)t].moddownConv; }
    // the relinearisation / rotation key a switch at ell limbs uses (its tier's when it has one)
    const DeviceBufferPtr& relinFor(uint32_t ell) const {
        const int t = tierAt(ell);
        return t >= 0 && tiers[(size_t)t].relinKey ? tiers[(size_t)t].relinKey : relinKey;
    }
    const DeviceBufferPtr* rotFor(uint32_t gal, uint32_t ell) const {
        const int t = tierAt(ell);
        if (t >= 0) {
            auto it = tiers[(size_t)t].rotKeys.find(gal);
            if (it != tiers[(size_t)t].rotKeys.end()) return &it->second;
        }
        auto it = rotKeys.find(gal);
        return it == rotKeys.end() ? nullptr : &it->second;
    }
    // bootstrapping precomputations per slot count (EvalBootstrapSetup)
    std::map<uint32_t, std::shared_ptr<BootstrapPrecomp>> boot;

    // memory pool (device words -> free list)
    std::mutex poolMu;
    // free lists per lane: a block freed on one lane is reused only by work
    // ordered after it (same lane, or any lane after a join)
    std::map<size_t, std::vector<uint64_t*>> freeList[SFP_MAX_LANES];
    std::vector<std::pair<size_t, uint64_t*>> deferredFree;  // cross-lane frees inside a region
    // batched ops (BeginBatch): their launches are issued at EndBatch, so a
    // block the batching thread frees while the batch is recorded is reused
    // only after it -- then by the ordinary rule (its lane and region, see
    // ~DeviceBuffer).  Blocks other threads free meanwhile take that rule at
    // once.  batchDepth / batchThread change under poolMu (buffers are freed
    // from any host thread).
    struct BatchFreed {
        size_t words;
        uint64_t* ptr;
        int lane;
        uint64_t region;
    };
    uint32_t batchDepth = 0;
    std::thread::id batchThread;
    std::vector<BatchFreed> batchFree;
    // a freed block back to the pool (poolMu held; `freer` = the freeing
    // thread's lane): private to its lane inside its region, deferred to the
    // join when another lane may still read it, lane 0's outside regions
    void poolReturn(size_t words, uint64_t* p, int lane, uint64_t region, int freer);
    // lane 0's free blocks at ForkLanes: every lane of the region is ordered
    // after them, so any lane may reuse them (without this, blocks a lane
    // allocates migrate to lane 0 at every join and the pool grows per region)
    std::map<size_t, std::vector<uint64_t*>> forkPool;
    int lane = 0;          // lane new work goes to
    int forkedLanes = 0;   // > 0 while a fork/join region is open
    uint64_t region = 0;   // id of the open region (0: none)
    uint64_t regionCount = 0;
    // cross-lane ordering: laneSeq[l] counts writes issued on lane l;
    // synced[h][x] = laneSeq[x] at the last time lane h waited for lane x
    uint64_t laneSeq[SFP_MAX_LANES] = {};
    uint64_t synced[SFP_MAX_LANES][SFP_MAX_LANES] = {};
    // SFHE_LANE_STATS (diagnostic): data-dependency waits (dep) issued inside
    // fork/join regions, printed at each JoinLanes
    uint64_t regionDepWaits = 0;
    void laneWait(int waiter, int waitee);
    int myLane() const;            // the calling thread's lane (0 unless SetLane)
    void setMyLane(int l);
    void dep(DeviceBuffer* b);     // current lane waits for b's last writer if needed
    void wrote(DeviceBuffer* b);   // b was just written on the current lane
    size_t poolBytes = 0;

    // serialises host-side use of the device from OpenMP callers
    std::recursive_mutex opMu;

    // plaintext encode cache (content -> device polynomial per level)
    bool ptCacheOn = true;
    size_t ptCacheBytes = 0;
    size_t ptCacheLimit = (size_t)48 << 30;
    std::unordered_map<uint64_t, std::vector<PtCacheEntry>> ptCache;  // key hash (incl. level)

    // graph capture: every block alloc() hands out while capturing (with its
    // size); blocks owned by a live graph are never recycled by the pool --
    // graphOwned[p] = true while a DeviceBuffer still holds p
    bool capturing = false;
    uint64_t captureEpoch = 0, epochCount = 0;  // id of the open capture (0: none)
    // >0: products inside the current region are formed canonically (lazy
    // rescaling held off; the Chebyshev PS evaluator, see chebyshev.cpp)
    uint32_t lazyHold = 0;
    std::set<uint64_t> abandonedEpochs;         // captures that were abandoned (their work never ran)
    std::vector<std::pair<uint64_t*, size_t>> capAllocs;
    std::unordered_map<uint64_t*, bool> graphOwned;

    std::atomic<uint64_t> seedCounter{1};
    uint64_t seed = 0;
    CryptoContextImpl<DCRTPoly>::OpStats stats;

    // limb sharding (one process per GPU): this rank holds Q limb i and P
    // limb k iff i % world == rank / k % world == rank, in increasing order,
    // so a ciphertext's local rows at any sharded level are a prefix of its
    // rows at level 0 and rescaling drops at most the last local row.
    // Tail replication: at levels with at most tailLimbs Q limbs every rank
    // holds and computes every row (no exchanges).  The
    // representation of a row set is a function of its limb count alone.
    // sharded is also set by a one-rank RCCL communicator: the sharded code
    // path (exchanges through RCCL) at W = 1, for single-GPU validation.
    int rank = 0, world = 1;
    // batch groups (EnableBatchGroups): this rank is in group bgroup of bgroups
    int bgroup = 0, bgroups = 1;
    bool bgatherAtOne = false;  // a one-group communicator still gathers (validation)
    bool sharded = false;
    uint32_t tailLimbs = 0;
    bool fullScope = false;  // inside FullScope: unsharded (setup work on every row)
    std::vector<DeviceBufferPtr> scopeKeep;  // uncached encodings alive until the scope ends
    // switching-key geometry: whole keys (rows 0), or this rank's slice of
    // every key (sfp_key_geom; set by EnableSharding)
    sfp_key_geom kgeom{};
    uint32_t keyRows() const { return kgeom.rows ? kgeom.rows : Lq + K; }
    std::map<uint32_t, std::vector<sfp_conv*>> modupConvShard;  // ell -> per digit (owned targets)
    // the same, split for the overlapped ModUp: per digit the
    // table of this rank's own source rows, then the whole digit with the
    // multipliers of those rows zeroed (the rows the all-gather brings)
    std::map<uint32_t, std::vector<std::pair<sfp_conv*, sfp_conv*>>> modupConvSplit;
    sfp_conv* moddownConvShard = nullptr;                        // P -> owned Q rows

    // ---- helpers ----
    uint32_t ellOf(uint32_t level) const { return Lq - level; }
    // scale of a product whose rescale to `level` is pending: Delta_level
    // times the prime that rescale drops (products of canonical operands at
    // level - 1 have exactly this scale: Delta_l^2 = Delta_{l+1} q)
    double preScale(uint32_t level) const { return scale[level] * (double)primes[ellOf(level)]; }
    // local rows among the first `count` limbs of a set dealt round-robin
    uint32_t owned(uint32_t count) const {
        return (uint32_t)rank < count ? (count - rank + world - 1) / world : 0;
    }
    // rows of ell limbs are dealt over the ranks (else every rank holds all)
    bool shardAt(uint32_t ell) const { return sharded && ell > tailLimbs; }
    uint32_t rows(uint32_t ell) const { return shardAt(ell) ? owned(ell) : ell; }  // local Q rows at ell limbs
    uint32_t prows(uint32_t ell) const { return shardAt(ell) ? owned(K) : K; }     // local P rows beside them
    // prime of local Q row i at ell limbs
    uint32_t qprime(uint32_t i, uint32_t ell) const { return shardAt(ell) ? rank + i * world : i; }
    uint32_t qprimeShard(uint32_t i) const { return rank + i * world; }
    sfp_limbs shardMap(uint32_t ell) const {  // this rank's dealt rows of ell limbs
        return sfp_limbs{owned(ell), owned(ell), 0, (uint32_t)rank, (uint32_t)world};
    }
    sfp_limbs qmap(uint32_t ell) const { return shardAt(ell) ? shardMap(ell) : sfp_limbs{ell, ell, 0, 0, 1}; }
    // local ext rows: the Q rows of ell limbs, then the P rows
    sfp_limbs extmap(uint32_t ell) const {
        return shardAt(ell) ? sfp_limbs{owned(ell) + owned(K), owned(ell), Lq + (uint32_t)rank, (uint32_t)rank,
                                        (uint32_t)world}
                            : sfp_limbs{ell + K, ell, Lq, 0, 1};
    }
    size_t polyWords(uint32_t level) const { return (size_t)rows(ellOf(level)) * n; }
    uint64_t nextSeed() { return seed ^ (0x9E3779B97F4A7C15ULL * (seedCounter++)); }
    DeviceBufferPtr alloc(size_t words);
    void releaseAll();
    void countBytes(double b) { stats.algo_bytes += b; }
};

// Setup work (key generation, encryption, decryption) runs on every row of a
// sharded context: inside this scope the state describes one rank holding all
// rows, and plaintext encodings are not cached (they would have the full rows).
class FullScope {
  public:
    explicit FullScope(SfheContextState* s)
        : s_(s), rank_(s->rank), world_(s->world), sharded_(s->sharded), was_(s->fullScope) {
        s->rank = 0;
        s->world = 1;
        s->sharded = false;
        s->fullScope = true;
    }
    ~FullScope() {
        s_->rank = rank_;
        s_->world = world_;
        s_->sharded = sharded_;
        s_->fullScope = was_;
        if (!was_) s_->scopeKeep.clear();  // later users of the blocks are stream-ordered after
    }

  private:
    SfheContextState* s_;
    int rank_, world_;
    bool sharded_, was_;
};

// Ops per batch (BeginBatch): SFHE_BATCH_WIDTH, 2..SFP_BATCH_MAX (default).
inline uint32_t batchWidth() {
    static const uint32_t w = [] {
        const char* v = std::getenv("SFHE_BATCH_WIDTH");
        const long x = v && *v ? std::strtol(v, nullptr, 10) : SFP_BATCH_MAX;
        return (uint32_t)std::max(2L, std::min<long>(x, SFP_BATCH_MAX));
    }();
    return w;
}

// Serialises host-side use of a context and routes the calling thread's
// operations to its lane (each host thread of a lane region has its own).
class OpLock {
  public:
    explicit OpLock(SfheContextState* s) : s_(s), g_(s->opMu) {
        s_->lane = s_->myLane();
        sfp_set_lane(s_->dev, s_->lane);
    }

  private:
    SfheContextState* s_;
    std::lock_guard<std::recursive_mutex> g_;
};

// splitmix64 (used for deterministic host sampling; identical in the oracle)
static inline uint64_t sf_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// CKKS special-FFT encoder (encoder.cpp)
// Returns shift >= 0: the coefficients are round(value * scale / 2^shift)
// (shift > 0 only when value * scale needs more than 62 bits); the caller
// multiplies the residues by 2^shift.
int ckks_encode(const std::vector<std::complex<double>>& v, uint32_t slots, uint32_t n,
                double scale, std::vector<int64_t>& coeffs);
void ckks_decode(const std::vector<double>& coeffs, uint32_t slots, uint32_t n,
                 std::vector<std::complex<double>>& out);
// the encoder's tables (rot[j] = 5^j mod 2n, ksi[k] = exp(2 pi i k / 2n) as
// (re, im) pairs), for the device encoder (sfp_encode_setup)
void ckks_encoder_tables(uint32_t n, const uint64_t** rot, const double** ksi);

}  // namespace lbcrypto
