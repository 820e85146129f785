// gfx950 (MI355X, CDNA4) implementation of the RNS primitive layer
// (csrc/prims.h).  All work is integer modular arithmetic on 64-bit
// residues of <= 60-bit primes: HBM-bound streaming kernels, no MFMA.
//
// Layout: a polynomial is `count` rows of n u64 (limb-major).  Every kernel
// maps (row, coefficient) -> thread with 16-byte per-lane accesses where the
// access is contiguous, so a wave moves 1 KiB per instruction.
//
// NTT: n = R * 256 is processed in two LDS-staged passes per limb:
//   column pass  - the first log2(R) Cooley-Tukey stages (strides >= 256)
//                  on tiles of R rows x (4096/R) columns;
//   row pass     - the last 8 stages (strides 128..1) on tiles of 16 rows
//                  of 256 contiguous words.
// Each pass reads and writes the limb once (2 HBM round trips per NTT).
// The inverse runs the mirrored Gentleman-Sande passes and folds 1/n into
// its last pass.  Twiddles are the bit-reversed psi tables (Shoup form).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_set>
#include <unordered_map>
#include <string>
#include <type_traits>
#include <vector>

#include "../modarith.h"
#include "../prims.h"

#define SFP_CHECK(call)                                                     \
    do {                                                                    \
        hipError_t e_ = (call);                                             \
        if (e_ != hipSuccess) record(d, #call, e_);                          \
    } while (0)

namespace {

constexpr int kThreads = 256;
constexpr int kTile = 4096;  // words per NTT tile (32 KiB of LDS)

struct Bar {
    u64 q, mu, r64;
    uint32_t b, pad;
};
static_assert(sizeof(Bar) == sizeof(sf_barrett), "layout");

__device__ __forceinline__ uint32_t primeOf(const sfp_limbs& m, uint32_t i) {
    const uint32_t st = m.stride ? m.stride : 1;
    return i < m.split ? m.base + i * st : m.pbase + (i - m.split) * st;
}

__device__ __forceinline__ u64 bmul(u64 a, u64 b, const sf_barrett& m) { return sf_mul(a, b, &m); }

__device__ __forceinline__ sf_barrett loadBar(const sf_barrett* t, uint32_t p) {
    sf_barrett m;
    m.q = t[p].q;
    m.mu = t[p].mu;
    m.r64 = t[p].r64;
    m.b = t[p].b;
    m.pad = 0;
    return m;
}

// 128-bit accumulator helpers
struct Acc {
    u64 lo, hi;
};
__device__ __forceinline__ void macc(Acc& a, u64 x, u64 y) {
    u64 l = x * y;
    u64 h = __umul64hi(x, y);
    u64 s = a.lo + l;
    a.hi += h + (s < l ? 1 : 0);
    a.lo = s;
}

}  // namespace

struct sfp_event {
    hipEvent_t e = nullptr;
    int lane = 0;
    uint64_t recId = 0;  // inside a stacked region: id of its latest (deferred) record
};

// One deferred item of a stacked region (sfp_stack_begin): a launch, or an
// event record / wait of a lane, issued in order by stackFlush.
struct StackRec {
    enum Kind : uint8_t { LAUNCH, EV_RECORD, EV_WAIT };
    Kind kind = LAUNCH;
    uint32_t cls = 0;  // merge class (STK_*; 0: always issued alone)
    uint64_t key = 0;  // two heads of one class and key may become one launch
    uint64_t id = 0;   // EV_RECORD: its id; EV_WAIT: the record it waits for (0: one before the region)
    sfp_event* ev = nullptr;
    uint32_t fam = ~0u;  // kernel family for live timing (sfp_prof_*), and its algorithmic bytes
    double bytes = 0;
    std::function<void(hipStream_t)> go;  // the launch on its own
    std::shared_ptr<void> pay;            // class payload (what stackMerge reads of both)
};

// A captured graph and the device arena its launches read their small
// argument arrays from (filled once, when the capture ends).
struct GraphChunk {
    u64* dev = nullptr;
    std::vector<u64> host;
    size_t used = 0;  // words
};
struct sfp_graph {
    hipGraph_t g = nullptr;
    hipGraphExec_t exec = nullptr;
    std::vector<GraphChunk> arena;
    std::unordered_map<uint64_t, std::vector<std::pair<std::vector<u64>, const u64*>>> consts;
    size_t nodes = 0;
    bool failed = false;
    std::string why;
};

struct sfp_dev {
    int device = 0;
    // lanes: independent in-order streams; every launch goes to streams[cur]
    hipStream_t streams[SFP_MAX_LANES] = {};
    int nLanes = 1, cur = 0;
    bool serial = false;  // sfp_serialize: every lane on streams[0]
    // stacked region (sfp_stack_begin): every lane's launches are recorded in
    // stack[lane] and issued by stackFlush on streams[0]; uploads and other
    // immediate stream work go to streams[0] directly (before the deferred
    // launches that read them)
    bool stackOn = false;
    std::vector<StackRec> stack[SFP_MAX_LANES];
    hipStream_t stackStream = nullptr;  // where the flush issues (null: streams[0])
    bool batchOn = false;               // a batched op (sfp_batch_begin): lists 4 + i
    int batchCur = 0;                   // the caller's lane (restored at sfp_batch_end)
    uint64_t recSeq = 0;
    std::vector<sfp_event*> stackFreedEv;  // freed inside the region: reusable after the flush
    uint64_t stkMerged = 0, stkSingle = 0;  // launches issued as merged pairs / alone
    sfp_key_geom kg = {};          // switching-key geometry (sfp_set_key_geom; rows 0: whole keys)
    uint32_t stkFam = ~0u;  // timedLaunch's family while it records (stacked)
    double stkBytes = 0;
    hipStream_t st() const {
        if (batchOn) return stackStream;
        return streams[(serial || stackOn) ? 0 : cur];
    }
    std::vector<sfp_event*> evFree;
    std::mutex evMu;  // evFree: buffers release events from any host thread
    uint32_t n = 0, logn = 0, np = 0;
    sf_barrett* bar = nullptr;  // device [np]
    u64 *psi = nullptr, *psiS = nullptr, *ipsi = nullptr, *ipsiS = nullptr;
    u64 *ninv = nullptr, *ninvS = nullptr;
    // FP64 twiddles for primes < 2^42 (exact doubles w and rounded w/q), and
    // per-prime 1/q and n^-1 as doubles
    double *psiD = nullptr, *ipsiD = nullptr;
    // ROW-pass row factors (rowTwLoad): [prime][k < 8][row < n/256] = psi_rev[row << k] (ipsi for irowD)
    double *rowD = nullptr, *irowD = nullptr;
    double *qinvD = nullptr, *ninvD = nullptr, *ninvQ = nullptr;
    std::vector<sf_barrett> hbar;
    std::vector<u64> hninv;  // n^-1 mod q per prime (ModUpPlan)
    std::map<const sfp_conv*, struct ModUpPlan*> plans;  // keyed by the level's digit-0 table
    // pinned argument ring (host) mirrored on the device
    char* hring = nullptr;
    char* dring = nullptr;
    size_t ringCap = 0, ringOff = 0;
    // pinned, host-coherent bounce buffer for bulk host<->device transfers
    // (read / written by kernels directly)
    char* bounce = nullptr;
    size_t bounceCap = 0;
    // live kernel timing (sfp_prof_*)
    struct ProfFam {
        uint32_t period = 0;
        uint64_t seen = 0, timed = 0;
        double ms = 0, bytes = 0;
        std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    } prof[SFP_FAM_COUNT];
    std::vector<hipEvent_t> evPool;
    // content-addressed device copies of small constant arrays (kernel
    // argument tables): bump-allocated in one buffer
    u64* cpool = nullptr;
    u64* cpoolOld = nullptr;  // the retired generation (devConst)
    size_t cpoolCap = 0, cpoolOff = 0;
    // contents -> pool offset; a miss is uploaded on the lane that made it
    // (stream-ordered, no drain), and another lane's first hit waits for
    // that upload's event
    struct ConstEntry {
        std::vector<u64> v;
        size_t off;
        int lane;
        hipEvent_t ev;
    };
    std::unordered_map<uint64_t, std::vector<ConstEntry>> cmap;
    std::mutex mu;
    std::string err;
    // limb sharding: this process is rank `rank` of `world`
    int rank = 0, world = 1;
    ncclComm_t nccl = nullptr;
    sfp_host_allgather_fn hostAg = nullptr;
    sfp_host_bcast_fn hostBc = nullptr;
    void* hostUser = nullptr;
    // batch groups (sfp_group_*): rank grank of gworld
    int grank = 0, gworld = 1;
    ncclComm_t gnccl = nullptr;
    sfp_host_allgather_fn gHostAg = nullptr;
    void* gHostUser = nullptr;
    // per-lane scratch (scratch()), and buffers retired by its growth
    std::mutex scrMu;
    u64* scr[SFP_MAX_LANES] = {};
    size_t scrWords[SFP_MAX_LANES] = {};
    std::vector<void*> retired;
    sfp_graph* capture = nullptr;  // open capture (sfp_capture_begin)
    // device CKKS encoder (sfp_encode): the host encoder's tables
    u64* encRot = nullptr;         // [n/2] 5^j mod 2n
    double2* encKsi = nullptr;     // [2n+1] exp(2 pi i k / 2n)
    // collective statistics (sfp_comm_stats): counts, bytes received, and
    // the event pairs of the timed (eager) collectives
    uint64_t commCalls = 0;
    double commBytes = 0;
    bool commTimed = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> commEv;
};

struct sfp_conv {
    uint32_t ns = 0, nt = 0;
    uint32_t* src = nullptr;  // device
    uint32_t* dst = nullptr;  // device
    u64* inv = nullptr;       // device [ns]
    u64* mod = nullptr;       // device [ns][nt]
    u64* sprod = nullptr;     // device [nt]: prod(S) mod dst_t (centred conversion)
    uint32_t* drow = nullptr; // device [nt]: output row of target t
    // FP64 form (k_convf / k_mdrsf; see ConvJob): targets split into FP64
    // and integer rows, FP64 multiplier tables over the FP64 targets
    bool fpOk = false;                       // at most kMaxConvBig 60-bit sources
    uint32_t nbig = 0;                       // 60-bit sources
    std::vector<uint32_t> hFpT, hIntT;       // ascending target indices
    uint32_t *fpT = nullptr, *intT = nullptr;
    // every target, ascending: the integer-only job of a table with more
    // 60-bit sources than the FP64 form splits (k_convf runs it on its
    // integer blocks)
    std::vector<uint32_t> hAll;
    uint32_t* allT = nullptr;
    double *invD = nullptr, *invQ = nullptr;  // [ns] inv as a double, inv / s_i
    double *vD = nullptr, *vQ = nullptr;      // [ns][hFpT.size()]
    double *hD = nullptr, *hQ = nullptr;      // [kMaxConvBig][hFpT.size()]
    std::vector<uint32_t> hsrc, hdst;
    std::vector<uint32_t> hrow;  // dst_row
    std::vector<u64> hinv, hmod; // host copies (ModUpPlan)
    // the fused ModDown COL pass's tables (k_moddown_col, built on first use):
    // mod[i][t] as a double and / q_t over every target, prod(S) mod q_t likewise
    double *mdD = nullptr, *mdQ = nullptr, *mdSpD = nullptr, *mdSpQ = nullptr;
    int mdState = 0;  // 0 not built, 1 built, -1 not eligible
};

struct ModUpPlan {
    uint32_t ell = 0, rows = 0;
    std::vector<const sfp_conv*> convs;
    u64 *postK = nullptr, *postKS = nullptr;
    double *postD = nullptr, *postQ = nullptr;
    double *mD = nullptr, *mQ = nullptr, *hD = nullptr, *hQ = nullptr;
    u64* mI = nullptr;
    bool big = false;
};
static void freePlan(ModUpPlan* P) {
    for (void* x : {(void*)P->postK, (void*)P->postKS, (void*)P->postD, (void*)P->postQ, (void*)P->mD, (void*)P->mQ,
                    (void*)P->hD, (void*)P->hQ, (void*)P->mI})
        hipFree(x);
    delete P;
}

static void record(sfp_dev* d, const char* what, hipError_t e) {
    std::lock_guard<std::mutex> g(d->mu);
    if (d->err.empty()) d->err = std::string(what) + ": " + hipGetErrorString(e);
}

static void captureFail(sfp_dev* d, const char* why) {
    if (!d->capture->failed) {
        d->capture->failed = true;
        d->capture->why = why;
    }
}

static void stackFlush(sfp_dev* d);

// A launch on the current lane: issued now, or recorded for the stacked
// region's flush (`launch` captures its arguments by value).
static void issue(sfp_dev* d, std::function<void(hipStream_t)>&& launch) {
    if (!d->stackOn) return launch(d->st());
    StackRec r;
    r.go = std::move(launch);
    r.fam = d->stkFam;
    r.bytes = d->stkBytes;
    d->stack[d->cur].push_back(std::move(r));
}
static void issueRec(sfp_dev* d, StackRec&& r) {
    if (!d->stackOn) return r.go(d->st());
    r.fam = d->stkFam;
    r.bytes = d->stkBytes;
    d->stack[d->cur].push_back(std::move(r));
}
#define SFP_GO(kern, grid, block, ...) \
    issue(d, [=](hipStream_t s_) { hipLaunchKernelGGL(kern, grid, block, 0, s_, __VA_ARGS__); })

// Drain every lane (shared host-visible resources: ring, bounce, constant pool).
static void syncAll(sfp_dev* d) {
    stackFlush(d);
    if (d->capture) return captureFail(d, "host synchronisation inside the captured region");
    for (int i = 0; i < d->nLanes; ++i) {
        hipError_t e = hipStreamSynchronize(d->streams[i]);
        if (e != hipSuccess) record(d, "synchronize", e);
    }
}

static bool debugSync() {
    static const bool on = [] {
        const char* v = std::getenv("SFHE_DEBUG_SYNC");
        return v && *v && *v != '0';
    }();
    return on;
}

static void checkLaunch(sfp_dev* d, const char* k) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) record(d, k, e);
    if (debugSync() && !d->capture && !d->stackOn) {
        e = hipStreamSynchronize(d->st());
        if (e != hipSuccess) record(d, k, e);
    }
}

// Every prime index a limb map can produce must exist: a kernel given an
// out-of-table prime would read garbage reduction constants (and a zero
// modulus never terminates a reduction loop), so reject the call on the host.
static bool limbsOk(sfp_dev* d, const sfp_limbs& m, const char* what) {
    if (!m.count) return true;
    uint32_t hi = 0;
    const uint32_t st = m.stride ? m.stride : 1;
    if (m.split) hi = m.base + (std::min(m.split, m.count) - 1) * st;
    if (m.count > m.split) hi = std::max(hi, m.pbase + (m.count - m.split - 1) * st);
    if (hi < d->np && m.count <= (1u << 20)) return true;
    std::lock_guard<std::mutex> g(d->mu);
    if (d->err.empty()) d->err = std::string(what) + ": limb map indexes past the prime table";
    return false;
}

// ---- live kernel timing ----
static hipEvent_t takeEvent(sfp_dev* d) {
    if (!d->evPool.empty()) {
        hipEvent_t e = d->evPool.back();
        d->evPool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    SFP_CHECK(hipEventCreate(&e));
    return e;
}

static void profFlush(sfp_dev* d, sfp_dev::ProfFam& f) {
    if (f.pending.empty()) return;
    SFP_CHECK(hipEventSynchronize(f.pending.back().second));
    for (auto& pr : f.pending) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) f.ms += ms;
        d->evPool.push_back(pr.first);
        d->evPool.push_back(pr.second);
    }
    f.pending.clear();
}

// Run `launch` (one kernel launch on d->st()); bracket it with events when
// this family is being timed and this launch is a sampled one.
template <class F>
static void timedLaunch(sfp_dev* d, uint32_t fam, double bytes, F&& launch) {
    sfp_dev::ProfFam& f = d->prof[fam];
    if (d->stackOn) {  // recorded: stackFlush times it as issued
        d->stkFam = fam;
        d->stkBytes = bytes;
        launch();
        d->stkFam = ~0u;
        d->stkBytes = 0;
        return;
    }
    if (d->capture || !f.period || (f.seen++ % f.period) != 0) {
        launch();
        return;
    }
    hipEvent_t a = takeEvent(d), b = takeEvent(d);
    SFP_CHECK(hipEventRecord(a, d->st()));
    launch();
    SFP_CHECK(hipEventRecord(b, d->st()));
    f.pending.push_back({a, b});
    f.timed++;
    f.bytes += bytes;
    if (f.pending.size() >= 8192) profFlush(d, f);
}

static unsigned gridFor(size_t work, unsigned perBlock) {
    size_t g = (work + perBlock - 1) / perBlock;
    return (unsigned)(g ? g : 1);
}

// ============================================================================
// NTT kernels

// One pass of the negacyclic NTT over 2048-word tiles.
//
// n = R * 256 is viewed as R rows of 256 words.  The forward transform is the
// bit-reversed-twiddle Cooley-Tukey schedule: global stage S (0..logn-1) pairs
// x with x + n/2^(S+1) and uses psi_rev[2^S + (x >> (logn - S))].
//   COL pass: stages 0..logR-1; a tile is C = 2048/R whole columns (R x C).
//   ROW pass: stages logR..logn-1; a tile is 8 whole rows (8 x 256).
// A block stages the tile in LDS (XOR-swizzled) with 16-byte coalesced loads
// and runs its stages in register rounds of up to LE stages: each thread pulls
// 2^LE words into registers, runs the round's radix-2 stages there and writes
// them back.  The tile size and LE were chosen by measurement (tools/
// microbench): a pass over few rows is latency-bound, so smaller tiles (more
// CUs) and more threads per tile win; 4096-word tiles or direct-from-HBM
// rounds were slower at every size.  Butterflies are lazy (Harvey):
// forward values live in [0, 4q), inverse values in [0, 2q); the pass that
// finishes the transform reduces to [0, q).  The inverse runs the
// Gentleman-Sande stages in reverse order (ROW pass first) and folds n^-1
// into the COL pass's store.
#ifndef SFHE_NTT_FP
#define SFHE_NTT_FP 1  // FP64 butterflies for primes < 2^42
#endif
#ifndef SFHE_NTT_TILE
#define SFHE_NTT_TILE 2048
#endif
constexpr int kNttTile = SFHE_NTT_TILE;         // words per tile (one block)
constexpr int kNttRows = kNttTile / 256;        // ROW pass: whole rows per tile
// LE = stages per register round (2^LE words per thread, kNttTile >> LE
// threads).  Launches below kNttSmallRows rows run LE = 2 (twice the waves per
// tile), larger ones LE = 3 (fewer rounds and barriers).  Measured on the
// sort (N=256 @ 2^16): thresholds 6 / 12 / 24 / 36 / all rows gave 64.6 / 63.8 /
// 63.3 / 62.5 / 62.2 ms, so every launch takes LE = 2 by default.
#ifndef SFHE_NTT_SMALL_ROWS
#define SFHE_NTT_SMALL_ROWS 4096
#endif
constexpr int kNttSmallRows = SFHE_NTT_SMALL_ROWS;

__device__ __forceinline__ uint32_t ldsSw(uint32_t e) {
    const uint32_t x = e >> 5;
    return e ^ ((x ^ (x << 2)) & 31u);
}
// ldsSw is linear over GF(2): for index bits that do not overlap,
// ldsSw(a | b) = ldsSw(a) ^ ldsSw(b).  A round's 2^B words of one thread sit at
// e0 | j*h*C (COL) or e0 | j*h (ROW), where e0 has zeros in j's bits, so
// their LDS slots are ldsSw(e0) ^ ldsSw(offset_j): one XOR per word, with
// offset_j a compile-time constant in the unrolled rounds.
template <bool COL>
__device__ __forceinline__ uint32_t ldsOff(uint32_t jh, uint32_t C) {
    return ldsSw(COL ? jh * C : jh);
}

struct NttTile {
    uint32_t logn, d;     // d = stages in this pass (logR or 8)
    uint32_t C, logC;     // COL: columns per tile (a power of two)
    uint32_t c0, r0;      // COL: first column; ROW: first row
};

// global index of tile-local sub-transform `st`, position u
template <bool COL>
__device__ __forceinline__ uint32_t nttGlobal(const NttTile& T, uint32_t st, uint32_t u) {
    return COL ? u * 256u + T.c0 + st : (T.r0 + st) * 256u + u;
}
template <bool COL>
__device__ __forceinline__ uint32_t nttLocal(const NttTile& T, uint32_t st, uint32_t u) {
    return COL ? u * T.C + st : st * 256u + u;
}

// Stage k of the pass (global stage S = S0 + k) at global index x0 uses
// psi_rev[2^S + (x0 >> (logn - S))].
//   COL (S0 = 0): x0 >> (logn - k) < 2^k: the pass needs only the table's
//       entries [1, 2^logR), shared by every tile -> staged in LDS once per
//       block (LDS word (2^k - 1) + ...), so its rounds never wait on HBM;
//   ROW (S0 = logR): 8 * 255 distinct entries per tile (twice the tile's own
//       bytes); staging them cost more occupancy than it saved, so the ROW
//       rounds read the table directly (index 2^S + (x0 >> (8 - k))).
constexpr uint32_t kNttColTw = 512;  // 2^logR - 1 entries, logR <= 9
template <bool COL>
__device__ __forceinline__ uint32_t twIndex(const NttTile& T, uint32_t S0, uint32_t k, uint32_t x0) {
    if (COL) return (1u << k) - 1 + (x0 >> (T.logn - k));
    return (1u << (S0 + k)) + (x0 >> (8 - k));
}
// One round: stages k0..k0+B-1 of the pass (k relative to the pass's first
// global stage S0).  8/2^B groups of 2^B words per thread.
template <bool INV, bool COL, int LE, int B, int TILE>
__device__ __forceinline__ void nttRound(u64* s, const NttTile& T, uint32_t S0, uint32_t k0, u64 q,
                                         const u64* w, const u64* wS) {
    constexpr int M = 1 << B;
    constexpr int GPT = (1 << LE) / M;  // groups per thread
    const uint32_t D = 1u << T.d;
    const uint32_t logh = T.d - k0 - B;
    const uint32_t h = 1u << logh;        // smallest stride of the round (in u)
    const uint32_t span = D >> k0;        // hi step
    const u64 q2 = 2 * q;
#pragma unroll
    for (int gi = 0; gi < GPT; ++gi) {
        const uint32_t gid = threadIdx.x + gi * (TILE >> LE);
        uint32_t st, lo, hi;
        if (COL) {  // every extent is a power of two: shifts and masks only
            st = gid & (T.C - 1);
            const uint32_t rest = gid >> T.logC;
            lo = rest & (h - 1);
            hi = rest >> logh;
        } else {
            lo = gid & (h - 1);
            const uint32_t rest = gid >> logh;
            hi = rest & ((1u << k0) - 1);
            st = rest >> k0;
        }
        const uint32_t ub = hi * span + lo;
        // stage t of the round uses psi_rev[2^S + (x0 >> (logn-S)) + (j >> (B-t))]
        // (x0 = member 0's global index): 2^t distinct twiddles (LDS)
        const uint32_t x0 = nttGlobal<COL>(T, st, ub);
        u64 W[M - 1], WS[M - 1];  // stage t's q-th twiddle at (1<<t)-1+q
#pragma unroll
        for (int t = 0; t < B; ++t) {
            const uint32_t tb = twIndex<COL>(T, S0, k0 + t, x0);
#pragma unroll
            for (int qd = 0; qd < (1 << t); ++qd) {
                W[(1 << t) - 1 + qd] = w[tb + qd];
                WS[(1 << t) - 1 + qd] = wS[tb + qd];
            }
        }
        u64 v[M];
        const uint32_t a0 = ldsSw(nttLocal<COL>(T, st, ub));
#pragma unroll
        for (int j = 0; j < M; ++j) v[j] = s[a0 ^ ldsOff<COL>(j * h, T.C)];
        if (!INV) {
            // Harvey CT butterfly: in [0,4q) -> out [0,4q)
#pragma unroll
            for (int t = 0; t < B; ++t) {
                const int half = 1 << (B - 1 - t);
#pragma unroll
                for (int j = 0; j < M; ++j) {
                    if (j & half) continue;
                    const int ti = (1 << t) - 1 + (j >> (B - t));
                    u64 X = v[j];
                    X = X >= q2 ? X - q2 : X;
                    const u64 Y = sf_mul_shoup_lazy(v[j + half], W[ti], WS[ti], q);
                    v[j] = X + Y;
                    v[j + half] = X - Y + q2;
                }
            }
        } else {
            // Harvey GS butterfly: in [0,2q) -> out [0,2q)
#pragma unroll
            for (int t = B - 1; t >= 0; --t) {
                const int half = 1 << (B - 1 - t);
#pragma unroll
                for (int j = 0; j < M; ++j) {
                    if (j & half) continue;
                    const int ti = (1 << t) - 1 + (j >> (B - t));
                    const u64 X = v[j], Y = v[j + half];
                    const u64 Sm = X + Y;
                    v[j] = Sm >= q2 ? Sm - q2 : Sm;
                    v[j + half] = sf_mul_shoup_lazy(X - Y + q2, W[ti], WS[ti], q);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < M; ++j) s[a0 ^ ldsOff<COL>(j * h, T.C)] = v[j];
    }
}

template <bool INV, bool COL, int LE, int TILE>
__device__ __forceinline__ void nttRoundDyn(int b, u64* s, const NttTile& T, uint32_t S0, uint32_t k0,
                                            u64 q, const u64* w, const u64* wS) {
    if constexpr (LE >= 4) {
        if (b == 4) return nttRound<INV, COL, LE, 4, TILE>(s, T, S0, k0, q, w, wS);
    }
    if constexpr (LE >= 3) {
        if (b == 3) return nttRound<INV, COL, LE, 3, TILE>(s, T, S0, k0, q, w, wS);
    }
    if (b == 2) return nttRound<INV, COL, LE, 2, TILE>(s, T, S0, k0, q, w, wS);
    nttRound<INV, COL, LE, 1, TILE>(s, T, S0, k0, q, w, wS);
}

// ---- FP64 butterflies (primes q < 2^42) ------------------------------------
// Residues are held as exact doubles.  For |Y| < 2^52, W in [0, q):
//   hi = Y*W, lo = fma(Y, W, -hi) (hi + lo == Y*W exactly),
//   qq = rint(Y * (W/q))            (within 1 of the true quotient),
//   r  = fma(-qq, q, hi) + lo       (exact: |hi - qq q| < 2^53)
// gives r == Y*W (mod q) with |r| < 2q.  Within one pass (<= 9 stages from
// [0, q)) forward values stay below 19q and inverse values below 2^9 q <
// 2^51, so no intermediate reduction is needed.
constexpr uint64_t kFpPrimeBound = 1ull << 42;

__device__ __forceinline__ double fpMulMod(double y, double w, double wq, double q) {
    const double hi = y * w;
    const double lo = fma(y, w, -hi);
    const double qq = rint(y * wq);
    return fma(-qq, q, hi) + lo;
}

// Exact u64 <-> double for integers below 2^52 (residues of primes < 2^42):
// the value rides in the mantissa of 2^52 + x, two VALU operations each
// instead of the generic 64-bit conversions' four to six.
__device__ __forceinline__ double u2d(u64 x) {
    return __longlong_as_double((long long)(x | 0x4330000000000000ull)) - 4503599627370496.0;
}
__device__ __forceinline__ u64 d2u(double v) {
    return (u64)__double_as_longlong(v + 4503599627370496.0) & 0x000FFFFFFFFFFFFFull;
}

// |v| < 2^52 -> [0, q)
__device__ __forceinline__ double fpReduce(double v, double q, double qinv) {
    double r = fma(-rint(v * qinv), q, v);
    return r < 0.0 ? r + q : r;
}

// PF: the round's 2^B - 1 twiddles were loaded into registers (pw) at the top
// of the kernel (ROW pass, see k_ntt), so the round does not wait on HBM.
// DC > 0: the pass's stage count is the compile-time DC (== T.d), so with an
// unrolled round loop every shift and mask below folds to a constant.
// W/q is formed from W in registers (half the twiddle bytes of a W/q table;
// a last-bit difference only moves the lazy quotient estimate by < 2^-6, and
// the outputs are canonical either way).
template <bool INV, bool COL, int LE, int B, int TILE, bool PF = false, int DC = 0>
__device__ __forceinline__ void nttRoundFP(double* s, const NttTile& T, uint32_t S0, uint32_t k0, double q,
                                           const double* w, double qinv, const double* pw = nullptr) {
    constexpr int M = 1 << B;
    constexpr int GPT = (1 << LE) / M;
    const uint32_t d = DC ? (uint32_t)DC : T.d;
    const uint32_t D = 1u << d;
    const uint32_t logh = d - k0 - B;
    const uint32_t h = 1u << logh;
    const uint32_t span = D >> k0;
    // COL columns per tile: TILE >> 8 when the pass's stage count is the
    // compile-time 8 (then the index math and every slot offset fold)
    const uint32_t Cc = (COL && DC == 8) ? (uint32_t)(TILE >> 8) : T.C;
    const uint32_t logCc = (COL && DC == 8) ? (uint32_t)__builtin_ctz(TILE >> 8) : T.logC;
#pragma unroll
    for (int gi = 0; gi < GPT; ++gi) {
        const uint32_t gid = threadIdx.x + gi * (TILE >> LE);
        uint32_t st, lo, hi;
        if (COL) {
            st = gid & (Cc - 1);
            const uint32_t rest = gid >> logCc;
            lo = rest & (h - 1);
            hi = rest >> logh;
        } else {
            lo = gid & (h - 1);
            const uint32_t rest = gid >> logh;
            hi = rest & ((1u << k0) - 1);
            st = rest >> k0;
        }
        const uint32_t ub = hi * span + lo;
        const uint32_t x0 = nttGlobal<COL>(T, st, ub);
        double W[M - 1], WQ[M - 1];
        if constexpr (PF) {
            static_assert(!COL && GPT == 1, "prefetched twiddles: ROW pass, one group per thread");
#pragma unroll
            for (int e = 0; e < M - 1; ++e) {
                W[e] = pw[e];
                WQ[e] = pw[e] * qinv;
            }
        } else {
#pragma unroll
            for (int t = 0; t < B; ++t) {
                const uint32_t tb = twIndex<COL>(T, S0, k0 + t, x0);
#pragma unroll
                for (int qd = 0; qd < (1 << t); ++qd) {
                    W[(1 << t) - 1 + qd] = w[tb + qd];
                    WQ[(1 << t) - 1 + qd] = W[(1 << t) - 1 + qd] * qinv;
                }
            }
        }
        double v[M];
        const uint32_t a0 = ldsSw(COL ? ub * Cc + st : st * 256u + ub);
#pragma unroll
        for (int j = 0; j < M; ++j) v[j] = s[a0 ^ ldsOff<COL>(j * h, Cc)];
        if (!INV) {
#pragma unroll
            for (int t = 0; t < B; ++t) {
                const int half = 1 << (B - 1 - t);
#pragma unroll
                for (int j = 0; j < M; ++j) {
                    if (j & half) continue;
                    const int ti = (1 << t) - 1 + (j >> (B - t));
                    const double X = v[j];
                    const double Y = fpMulMod(v[j + half], W[ti], WQ[ti], q);
                    v[j] = X + Y;
                    v[j + half] = X - Y;
                }
            }
        } else {
#pragma unroll
            for (int t = B - 1; t >= 0; --t) {
                const int half = 1 << (B - 1 - t);
#pragma unroll
                for (int j = 0; j < M; ++j) {
                    if (j & half) continue;
                    const int ti = (1 << t) - 1 + (j >> (B - t));
                    const double X = v[j], Y = v[j + half];
                    v[j] = X + Y;
                    v[j + half] = fpMulMod(X - Y, W[ti], WQ[ti], q);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < M; ++j) s[a0 ^ ldsOff<COL>(j * h, Cc)] = v[j];
    }
}

template <bool INV, bool COL, int LE, int TILE>
__device__ __forceinline__ void nttRoundDynFP(int b, double* s, const NttTile& T, uint32_t S0, uint32_t k0,
                                              double q, const double* w, double qinv) {
    if constexpr (LE >= 4) {
        if (b == 4) return nttRoundFP<INV, COL, LE, 4, TILE>(s, T, S0, k0, q, w, qinv);
    }
    if constexpr (LE >= 3) {
        if (b == 3) return nttRoundFP<INV, COL, LE, 3, TILE>(s, T, S0, k0, q, w, qinv);
    }
    if (b == 2) return nttRoundFP<INV, COL, LE, 2, TILE>(s, T, S0, k0, q, w, qinv);
    nttRoundFP<INV, COL, LE, 1, TILE>(s, T, S0, k0, q, w, qinv);
}


// ROW-pass FP64 twiddles of one thread (LE = 2: four rounds x three).  Stage
// k of the pass at row `row` and in-row offset v uses psi_rev[2^S + row 2^k + v]
// (S = S0 + k, v < 2^k): across the pass, all n entries of the table, 8 B per
// coefficient on top of the tile's 16.  The bit-reversed exponent of that
// index is the sum of those of its disjoint bit fields, so the twiddle is also
//   psi_rev[2^S + v] * psi_rev[row 2^k]  (mod q):
// a local factor (2^k entries per stage, shared by every row of the prime:
// cache-resident) times the row factor rowD[k][row] (wave-uniform: scalar
// loads).  The last round (stages 6 and 7, three quarters of the table) takes
// its three twiddles that way, as exact products (fpMulMod, |W| < 1.5 q: W
// only multiplies, outputs stay canonical and bit-identical); rounds 0-2 read
// the table (factoring them too cost more VALU time than their bytes).
struct RowTw {
    double L[12];
    double R[2];
};
__device__ __forceinline__ void rowTwIssue(RowTw& W, const double* __restrict__ gd, const double* __restrict__ rd,
                                           const NttTile& T, uint32_t S0) {
    const uint32_t gid = threadIdx.x;
    const uint32_t row = __builtin_amdgcn_readfirstlane(T.r0 + (gid >> 6));  // (st = gid >> 6 every round)
    const uint32_t rowsLog = __builtin_amdgcn_readfirstlane(T.logn - 8);
#pragma unroll
    for (int t = 0; t < 2; ++t) W.R[t] = rd[((uint32_t)(6 + t) << rowsLog) + row];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t k0 = 2 * r, logh = 8 - k0 - 2;
        const uint32_t lo = gid & ((1u << logh) - 1);
        const uint32_t hi = (gid >> logh) & ((1u << k0) - 1);
        const uint32_t u = hi * (256u >> k0) + lo;
        const uint32_t x0 = (T.r0 + (gid >> 6)) * 256u + u;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint32_t k = k0 + t;
            const uint32_t b = r == 3 ? (1u << (S0 + k)) + (u >> (8 - k)) : (1u << (S0 + k)) + (x0 >> (8 - k));
#pragma unroll
            for (int qd = 0; qd < (1 << t); ++qd) W.L[3 * r + (1 << t) - 1 + qd] = gd[b + qd];
        }
    }
}
__device__ __forceinline__ void rowTwFinish(double* PW, const RowTw& W, double q, double qi) {
#pragma unroll
    for (int i = 0; i < 9; ++i) PW[i] = W.L[i];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const double rf = W.R[t], rfq = rf * qi;
#pragma unroll
        for (int qd = 0; qd < (1 << t); ++qd) {
            const int i = 9 + (1 << t) - 1 + qd;
            PW[i] = fpMulMod(W.L[i], rf, rfq, q);
        }
    }
}

// A 2-D set of rows for one NTT launch, passed by value: row (p, i) for
// p < P, i < R lives at base + p*ps + i*is (word offsets).  Prime of row i:
// primeOf(pm, i).  The first pass reads `src` (optionally the centred lift of
// a row modulo prime `liftPrime`; optionally also writing the raw words to
// `copy`), the intermediate lands in `dst`, and the last pass writes `dst` --
// or, with `epi`, eout = (ein - v) * k_i (+ eout when `add`).
struct RowPtr {
    const u64* base;
    long long ps, is;  // word strides (may be negative: two unrelated buffers)
};
struct RowGroup {
    uint32_t P, R;
    sfp_limbs pm;
    RowPtr src, dst, copy, ein, eout;
    uint32_t copyByAlpha;  // copy row = copy.base + (i / alpha) * ps + i * is
    uint32_t alpha;
    uint32_t skipEll;      // >0: skip rows alpha*p <= i < min(alpha*(p+1), skipEll) (ModUp own digit)
    uint32_t lift, liftPrime;
    uint32_t epi, addMask;  // addMask bit p: accumulate into eout for polynomial p
    RowPtr eadd;            // epi with eadd.base: eout += eadd * k2_i
    // epi with tA0: eadd is the tensor product of (tA0, tA1) and (tB0, tB1)
    // formed here (row i, n words per row): a0 b0 for polynomial 0, a0 b1 +
    // a1 b0 for polynomial 1 (sfp_mult_relin_rescale: the tensor is never
    // written out)
    const u64 *tA0, *tA1, *tB0, *tB1;
    // multipliers (a rescale fused with the product before it):
    //   pre / preK: the first pass reads src * pre (elementwise) or src * preK_i
    //   emul / emK: the epilogue uses ein * emul or ein * emK_i in place of ein
    RowPtr pre, emul;
    // device arrays (constant cache): epilogue constants per i (value, Shoup)
    // and q_liftPrime mod q_i -- pointers keep the kernel arguments small
    const u64 *k, *kS, *k2, *k2S, *liftSub, *preK, *preKS, *emK, *emKS;
    // ModUp's conversion fused into the forward COL pass (k_ntt<..., CONV>,
    // ModUpPlan): row (p, i) is Conv_p(y)_i = sum_s y_{p,s} m_p[s][i] mod q_i,
    // read from the digit's source rows y (cy + (p alpha + s) n: FP64 rows as
    // doubles, the 60-bit q_0 as u64) instead of its own row.  Multipliers
    // [p][s][i] (stride cRows): cmD / cmQ (as double, / q_i) for FP64 rows,
    // cmI for integer rows; chD / chQ [i]: q_0's high-part multiplier (cBig)
    const u64* cy;
    const double *cmD, *cmQ, *chD, *chQ;
    const u64* cmI;
    uint32_t cRows, cBig;
    // inverse COL pass: scale row i by post_i (n^-1 times the conversion's
    // source factor) instead of n^-1; FP64 rows are stored as doubles
    const u64 *postK, *postKS;
    const double *postD, *postQ;
    // ModDown's conversion fused into the forward COL pass (k_moddown_col):
    // the per-level table (device); the call's rows ride in fields the
    // forward pass's first half otherwise uses: copy = the K source (P) rows
    // of polynomial p, coefficient form; pre = its dropped row l (with rescale)
    const struct MdColArgs* md;
    // icol (k_ntt<false, true, ..., ICOL>, with lift): src is the dropped row
    // after only the FIRST pass of its inverse NTT (the ROW pass); the forward
    // COL pass runs the inverse COL pass of that tile (prime liftPrime,
    // inverse twiddles iTw / iTwS / iTwD, n^-1) in its prologue, then lifts:
    // a rescale's dropped row never makes the inverse COL round trip
    uint32_t icol;
    const u64 *iTw, *iTwS;
    const double* iTwD;
};

// Merged launches (stacked regions, batched ops; sfp_stack_begin /
// sfp_batch_begin): NG independent argument sets in one launch.  Set i owns
// the grid rows [start[i], start[i+1]) (renumbered from 0); with `inter` (NG
// sets of equal row counts) the sets alternate instead -- grid row y is row
// y / NG of set y % NG -- so the sets' rows of one prime (one key row, one
// twiddle table) run side by side and share their L2 lines.  NG = 1 is the
// ordinary launch.
template <class T, int NG>
struct ArgSet {
    T a[NG];
    uint32_t start[NG];  // start[0] = 0
    uint32_t inter;
};
template <class T, int NG>
__device__ __forceinline__ uint32_t argSel(const ArgSet<T, NG>& S, uint32_t& row) {
    const uint32_t y = blockIdx.y;
    if (NG == 1) {
        row = y;
        return 0;
    }
    if (S.inter) {
        row = y / NG;
        return y % NG;
    }
    uint32_t sel = 0;
#pragma unroll
    for (int i = 1; i < NG; ++i)
        if (y >= S.start[i]) sel = (uint32_t)i;
    row = y - S.start[sel];
    return sel;
}
template <int NG>
using RowGroupSet = ArgSet<RowGroup, NG>;

__device__ __forceinline__ u64* rowAt(const RowPtr& r, uint32_t p, uint32_t i) {
    return const_cast<u64*>(r.base) + p * r.ps + i * r.is;
}

// Developer build knob: SFHE_NTT_TRACE accumulates per-phase shader clocks
// of every block (thread 0, after each barrier) for tools/microbench.  The
// deltas stay in registers until the block's end (an atomic per mark would be
// waited for by the next barrier and inflate the phase it ends).
#ifdef SFHE_NTT_TRACE
constexpr int kTraceSlots = 256;  // spread the atomics: no contention artefacts
__device__ unsigned long long g_nttTrace[kTraceSlots][4][8];
__device__ unsigned long long g_mdrsTrace[kTraceSlots][8];  // k_mdrsf (FP64 blocks): phases 0..3, [7] blocks
#define NTT_MARK(i)                                                          \
    {                                                                        \
        const unsigned long long t_ = clock64();                             \
        tacc[(i)] += t_ - tprev;                                             \
        tprev = t_;                                                          \
    }
#else
#define NTT_MARK(i)
#endif

template <bool INV, bool COL, int LE, int TILE, int NG = 1, bool CONV = false, bool ICOL = false>
__global__ __launch_bounds__(TILE >> LE) void k_ntt(const RowGroupSet<NG> GS, const sf_barrett* __restrict__ bar,
                                                  const u64* __restrict__ tw, const u64* __restrict__ twS,
                                                  const u64* __restrict__ ninv,
                                                  const u64* __restrict__ ninvS, uint32_t logn,
                                                  const double* __restrict__ twD,
                                                  const double* __restrict__ qinvD,
                                                  const double* __restrict__ ninvD,
                                                  const double* __restrict__ ninvQ, int useFp,
                                                  const double* __restrict__ rowD) {
    __shared__ u64 s[TILE];
    __shared__ u64 tW[COL ? kNttColTw : 1], tX[COL ? kNttColTw : 1];  // COL twiddles (value; Shoup for integer rows)
    __shared__ u64 tWi[ICOL ? kNttColTw : 1], tXi[ICOL ? kNttColTw : 1];  // ICOL: the source row's inverse ones
    static_assert(!ICOL || (!INV && COL && !CONV), "the inverse COL prologue feeds the forward COL pass");
#ifdef SFHE_NTT_TRACE
    unsigned long long tprev = clock64(), tacc[6] = {0, 0, 0, 0, 0, 0};
#endif
    constexpr bool FIRST = (COL != INV);  // forward: COL first; inverse: ROW first
    const uint32_t n = 1u << logn;
    const uint32_t logR = logn - 8;
    uint32_t rid;
    const RowGroup& G = GS.a[argSel(GS, rid)];
    const uint32_t pp = rid / G.R, ii = rid % G.R;
    if (G.skipEll && ii >= G.alpha * pp && ii < min(G.alpha * (pp + 1), G.skipEll)) return;
    const uint32_t prime = primeOf(G.pm, ii);
    NttTile T;
    T.logn = logn;
    T.d = COL ? logR : 8u;
    T.logC = COL ? (uint32_t)__builtin_ctz(TILE) - logR : 0u;
    T.C = 1u << T.logC;
    // XCD-aware tile order: workgroups go to the 8 XCDs round-robin by id, so
    // block x runs on XCD x % 8.  Give each XCD a contiguous run of tiles:
    // COL tiles of C < 16 words share 128-byte lines with their neighbours
    // (and ROW tiles share twiddle lines), which then meet in one L2.
    const uint32_t tile = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    T.c0 = COL ? tile * T.C : 0u;
    T.r0 = COL ? 0u : tile * (TILE / 256);
    const uint32_t S0 = COL ? 0u : logR;
    constexpr int NT = TILE >> LE, NPAIR = (1 << LE) / 2;

    // Every global load the prologue needs is issued before the first wait:
    // the tile (and its pre-multiplier), both
    // twiddle forms (the row's arithmetic is known only once q arrives), then
    // the prime.  One HBM round trip instead of one per dependent step.
    const u64* in = FIRST ? rowAt(G.src, pp, ii) : rowAt(G.dst, pp, ii);
    const u64* pre = FIRST && G.pre.base ? rowAt(G.pre, pp, ii) : nullptr;
    const bool epi = !FIRST && G.epi;
    const u64* ein = epi ? rowAt(G.ein, pp, ii) : nullptr;
    auto tileOff = [&](int k) -> size_t {
        const uint32_t e = 2 * (threadIdx.x + k * NT);
        return COL ? (size_t)(e >> T.logC) * 256 + T.c0 + (e & (T.C - 1)) : (size_t)T.r0 * 256 + e;
    };
    ulonglong2 xr[NPAIR], mr[NPAIR];
    if constexpr (CONV) {
        static_assert(!INV && COL, "the conversion feeds the forward COL pass");
        // this tile of Conv_pp(y) for target row ii (ModUp): the digit's
        // source tiles come in groups of four (loads in flight together; the
        // sources were read by the other target rows' blocks too: L2 hits)
        const uint32_t ns = min(G.alpha, G.skipEll - pp * G.alpha);
        const u64* yb = G.cy + (size_t)pp * G.alpha * n;
        const size_t tb = (size_t)pp * G.alpha * G.cRows + ii;
        const u64 qc = bar[prime].q;
        const bool big0 = G.cBig && pp == 0;
        constexpr int GRP = 4;
        if (useFp && qc < kFpPrimeBound) {
            const double qd = (double)qc, qi = qinvD[prime];
            double acc[2 * NPAIR];
#pragma unroll
            for (int w = 0; w < 2 * NPAIR; ++w) acc[w] = 0.0;
            for (uint32_t s0 = 0; s0 < ns; s0 += GRP) {
                ulonglong2 v[GRP][NPAIR];
#pragma unroll
                for (int g = 0; g < GRP; ++g)
                    if (s0 + g < ns)
#pragma unroll
                        for (int k = 0; k < NPAIR; ++k)
                            v[g][k] = *reinterpret_cast<const ulonglong2*>(yb + (size_t)(s0 + g) * n + tileOff(k));
#pragma unroll
                for (int g = 0; g < GRP; ++g) {
                    const uint32_t sI = s0 + g;
                    if (sI >= ns) break;
                    const double md = G.cmD[tb + (size_t)sI * G.cRows], mq = G.cmQ[tb + (size_t)sI * G.cRows];
                    if (big0 && sI == 0) {  // y < 2^60: y_lo + 2^30 y_hi, the second with mod 2^30 mod q
                        const double hd = G.chD[ii], hq = G.chQ[ii];
#pragma unroll
                        for (int k = 0; k < NPAIR; ++k) {
                            const u64 ya = v[g][k].x, yc = v[g][k].y;
                            acc[2 * k] += fpMulMod(u2d(ya & 0x3fffffffull), md, mq, qd) +
                                          fpMulMod(u2d(ya >> 30), hd, hq, qd);
                            acc[2 * k + 1] += fpMulMod(u2d(yc & 0x3fffffffull), md, mq, qd) +
                                              fpMulMod(u2d(yc >> 30), hd, hq, qd);
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < NPAIR; ++k) {
                            acc[2 * k] += fpMulMod(__longlong_as_double(v[g][k].x), md, mq, qd);
                            acc[2 * k + 1] += fpMulMod(__longlong_as_double(v[g][k].y), md, mq, qd);
                        }
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {  // |acc| < 14 * 1.5 q < 2^46: exact
                xr[k].x = d2u(fpReduce(acc[2 * k], qd, qi));
                xr[k].y = d2u(fpReduce(acc[2 * k + 1], qd, qi));
            }
        } else {  // an integer target row (q_0 for digits > 0): 128-bit sums of canonical residues
            const sf_barrett CB = loadBar(bar, prime);
            Acc acc[2 * NPAIR];
#pragma unroll
            for (int w = 0; w < 2 * NPAIR; ++w) acc[w] = Acc{0, 0};
            for (uint32_t sI = 0; sI < ns; ++sI) {
                const u64 m = G.cmI[tb + (size_t)sI * G.cRows];
                const bool raw = big0 && sI == 0;
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {
                    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(yb + (size_t)sI * n + tileOff(k));
                    macc(acc[2 * k], raw ? v.x : d2u(__longlong_as_double(v.x)), m);
                    macc(acc[2 * k + 1], raw ? v.y : d2u(__longlong_as_double(v.y)), m);
                }
            }
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {
                xr[k].x = sf_reduce128_acc(acc[2 * k].lo, acc[2 * k].hi, &CB);
                xr[k].y = sf_reduce128_acc(acc[2 * k + 1].lo, acc[2 * k + 1].hi, &CB);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) xr[k] = *reinterpret_cast<const ulonglong2*>(in + tileOff(k));
    }
    if (pre) {
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) mr[k] = *reinterpret_cast<const ulonglong2*>(pre + tileOff(k));
    }
    const u64* gwI = tw + (size_t)prime * n;
    const u64* gwD = reinterpret_cast<const u64*>(twD) + (size_t)prime * n;
    const u64* gx = twS + (size_t)prime * n;
    // COL: twiddle entries [1, 2^logR) -> LDS (clamped indices: unconditional loads)
    constexpr int kColPer = COL ? (int)((kNttColTw + NT - 1) / NT) : 1;
    const uint32_t colTw = (1u << logR) - 1;
    u64 cwI[kColPer], cwX[kColPer], cwD[kColPer];
    if (COL) {
#pragma unroll
        for (int c = 0; c < kColPer; ++c) {
            const uint32_t e = min(threadIdx.x + c * NT, colTw - 1) + 1;
            cwI[c] = gwI[e];
            cwX[c] = gx[e];
            cwD[c] = gwD[e];
        }
    }
    // ICOL: the source row's prime and its inverse COL-pass twiddles, in
    // flight with the tile and the forward ones
    const uint32_t lp = ICOL ? G.liftPrime : 0u;
    u64 icI[ICOL ? kColPer : 1], icX[ICOL ? kColPer : 1], icD[ICOL ? kColPer : 1];
    if constexpr (ICOL) {
        const u64* iI = G.iTw + (size_t)lp * n;
        const u64* iX = G.iTwS + (size_t)lp * n;
        const u64* iD = reinterpret_cast<const u64*>(G.iTwD) + (size_t)lp * n;
#pragma unroll
        for (int c = 0; c < kColPer; ++c) {
            const uint32_t e = min(threadIdx.x + c * NT, colTw - 1) + 1;
            icI[c] = iI[e];
            icX[c] = iX[e];
            icD[c] = iD[e];
        }
    }
    // ROW pass, FP64 rows, one group per thread per round (LE = 2): every
    // round's twiddles are data-independent, so all 4 x 3 of them (as local
    // and row factors, rowTwIssue) are loaded here, in flight together with
    // the tile, instead of one latency per register round
    constexpr bool kPfBuild = !COL && LE == 2;
    constexpr int kPfRounds = 8 / 2;
    double PW[kPfBuild ? kPfRounds * 3 : 1];
    RowTw RT;
    if constexpr (kPfBuild)
        rowTwIssue(RT, reinterpret_cast<const double*>(gwD), rowD + (size_t)prime * 8 * (n >> 8), T, S0);
    sf_barrett LB{};
    u64 lsub = 0;
    const bool preK = FIRST && G.preK;
    const u64 pk = preK ? G.preK[ii] : 0, pkS = preK ? G.preKS[ii] : 0;
    if (FIRST && (G.lift || pre)) LB = loadBar(bar, prime);
    if (FIRST && G.lift) lsub = G.liftSub[ii];
    const u64 lhalf = (FIRST && G.lift) ? (bar[G.liftPrime].q >> 1) : 0;
    const u64 q = bar[prime].q;
    const bool fp = useFp && q < kFpPrimeBound;  // uniform per block
    const bool rowPf = kPfBuild && fp;
    if constexpr (kPfBuild)
        if (rowPf) rowTwFinish(PW, RT, (double)q, qinvD[prime]);

    // the pass's twiddle table for this prime: FP64 values (W/q is formed in
    // registers) or integer values with their Shoup companions
    const u64* gw = fp ? gwD : gwI;
    if (COL) {
#pragma unroll
        for (int c = 0; c < kColPer; ++c) {
            const uint32_t e = threadIdx.x + c * NT;
            if (e < colTw) {
                tW[e] = fp ? cwD[c] : cwI[c];
                if (!fp) tX[e] = cwX[c];
            }
        }
    }
    const u64 qL = ICOL ? bar[lp].q : 0;
    const bool fpL = ICOL && useFp && qL < kFpPrimeBound;  // the source row's arithmetic
    if constexpr (ICOL) {
#pragma unroll
        for (int c = 0; c < kColPer; ++c) {
            const uint32_t e = threadIdx.x + c * NT;
            if (e < colTw) {
                tWi[e] = fpL ? icD[c] : icI[c];
                if (!fpL) tXi[e] = icX[c];
            }
        }
    }
    const u64* rw = COL ? tW : gw;
    const u64* rx = COL ? tX : gx;
    u64* cp = nullptr;
    if (FIRST && G.copy.base)
        cp = G.copyByAlpha ? const_cast<u64*>(G.copy.base) + (ii / G.alpha) * G.copy.ps + ii * G.copy.is
                           : rowAt(G.copy, pp, ii);

    // tile -> LDS, 16 B per lane; tile-linear word e is row-major (u, st)
#pragma unroll
    for (int k = 0; k < NPAIR; ++k) {
        const uint32_t e = 2 * (threadIdx.x + k * NT);
        const size_t g = tileOff(k);
        ulonglong2 x = xr[k];
        if constexpr (ICOL) {  // the source row as its own prime's pass stages it (lifted after its COL rounds)
            s[ldsSw(e)] = fpL ? __double_as_longlong(u2d(x.x)) : x.x;
            s[ldsSw(e + 1)] = fpL ? __double_as_longlong(u2d(x.y)) : x.y;
            continue;
        }
        if (FIRST) {
            if (cp) *reinterpret_cast<ulonglong2*>(cp + g) = x;
            if (pre) {
                const ulonglong2 m = mr[k];
                x.x = bmul(x.x, m.x, LB);
                x.y = bmul(x.y, m.y, LB);
            }
            if (preK) {
                x.x = sf_mul_shoup(x.x, pk, pkS, q);
                x.y = sf_mul_shoup(x.y, pk, pkS, q);
            }
            if (G.lift) {
                u64 r0 = sf_reduce128(x.x, 0, &LB), r1 = sf_reduce128(x.y, 0, &LB);
                if (x.x > lhalf) r0 = sf_sub(r0, lsub, q);
                if (x.y > lhalf) r1 = sf_sub(r1, lsub, q);
                x.x = r0;
                x.y = r1;
            }
        }
        if (fp) {
            s[ldsSw(e)] = __double_as_longlong(u2d(x.x));
            s[ldsSw(e + 1)] = __double_as_longlong(u2d(x.y));
        } else {
            s[ldsSw(e)] = x.x;
            s[ldsSw(e + 1)] = x.y;
        }
    }
    __syncthreads();
    NTT_MARK(0);
    const uint32_t nr = (T.d + LE - 1) / LE;
    if constexpr (ICOL) {
        // the source tile's inverse COL pass (k_ntt<true, true>'s rounds and
        // its n^-1 store, canonical mod q_l) ...
        const double qLd = (double)qL, qLi = qinvD[lp];
        for (uint32_t ri = 0; ri < nr; ++ri) {
            const uint32_t r = nr - 1 - ri;
            const uint32_t k0 = LE * r;
            const int b = (int)min((uint32_t)LE, T.d - k0);
            if (fpL)
                nttRoundDynFP<true, true, LE, TILE>(b, reinterpret_cast<double*>(s), T, 0u, k0, qLd,
                                                    reinterpret_cast<const double*>(tWi), qLi);
            else
                nttRoundDyn<true, true, LE, TILE>(b, s, T, 0u, k0, qL, tWi, tXi);
            __syncthreads();
        }
        // ... then, word by word (each thread its own slots), the centred lift
        // to this row's prime that the unfused forward pass applies at its load
        const u64 niL = ninv[lp], niLS = ninvS[lp];
        const double niLD = ninvD[lp], niLQ = ninvQ[lp];
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) {
            const uint32_t e = 2 * (threadIdx.x + k * NT);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                u64 v = s[ldsSw(e + h)];
                if (fpL) {
                    v = d2u(fpReduce(fpMulMod(__longlong_as_double(v), niLD, niLQ, qLd), qLd, qLi));
                } else {
                    v = sf_mul_shoup_lazy(v, niL, niLS, qL);
                    v = v >= qL ? v - qL : v;
                }
                u64 rr = sf_reduce128(v, 0, &LB);
                if (v > lhalf) rr = sf_sub(rr, lsub, q);
                s[ldsSw(e + h)] = fp ? __double_as_longlong(u2d(rr)) : rr;
            }
        }
        __syncthreads();
    }
    if constexpr (kPfBuild) {
        if (rowPf) {
#pragma unroll
            for (int ri = 0; ri < kPfRounds; ++ri) {
                const int r = INV ? kPfRounds - 1 - ri : ri;
                nttRoundFP<INV, false, 2, 2, TILE, true, 8>(reinterpret_cast<double*>(s), T, S0, 2 * r,
                                                            (double)q, nullptr, qinvD[prime], PW + 3 * r);
                __syncthreads();
                NTT_MARK(1 + ri);
            }
        }
    }
    // COL pass over 2^8 rows (ring 2^16), FP64 rows, LE = 2: the same four
    // rounds unrolled with compile-time strides (twiddles already in LDS).
    constexpr bool kColUnrollBuild = COL && LE == 2;
    const bool colUnroll = kColUnrollBuild && fp && T.d == 8u;
    if constexpr (kColUnrollBuild) {
        if (colUnroll) {
#pragma unroll
            for (int ri = 0; ri < 4; ++ri) {
                const int r = INV ? 3 - ri : ri;
                nttRoundFP<INV, true, 2, 2, TILE, false, 8>(reinterpret_cast<double*>(s), T, S0, 2 * r, (double)q,
                                                            reinterpret_cast<const double*>(rw), qinvD[prime]);
                __syncthreads();
                NTT_MARK(1 + ri);
            }
        }
    }
    for (uint32_t ri = 0; ri < ((rowPf || colUnroll) ? 0u : nr); ++ri) {
        const uint32_t r = INV ? nr - 1 - ri : ri;
        const uint32_t k0 = LE * r;
        const int b = (int)min((uint32_t)LE, T.d - k0);
        if (fp)
            nttRoundDynFP<INV, COL, LE, TILE>(b, reinterpret_cast<double*>(s), T, S0, k0, (double)q,
                                              reinterpret_cast<const double*>(rw), qinvD[prime]);
        else
            nttRoundDyn<INV, COL, LE, TILE>(b, s, T, S0, k0, q, rw, rx);
        __syncthreads();
        NTT_MARK(1 + ri);
    }
    const bool scale = INV && COL;
    const bool post = scale && G.postK;  // (ModUpPlan: n^-1 times the conversion's source factor)
    const u64 ni = post ? G.postK[ii] : scale ? ninv[prime] : 0, niS = post ? G.postKS[ii] : scale ? ninvS[prime] : 0;
    u64* out = epi ? rowAt(G.eout, pp, ii) : rowAt(G.dst, pp, ii);
    const u64 ek = epi ? G.k[ii] : 0, ekS = epi ? G.kS[ii] : 0;
    const u64* ead = epi && G.eadd.base ? rowAt(G.eadd, pp, ii) : nullptr;
    const bool tens = epi && G.tA0;
    const u64 ek2 = (ead || tens) ? G.k2[ii] : 0, ek2S = (ead || tens) ? G.k2S[ii] : 0;
    const u64* emul = epi && G.emul.base ? rowAt(G.emul, pp, ii) : nullptr;
    const bool emK = epi && G.emK;
    const u64 emk = emK ? G.emK[ii] : 0, emkS = emK ? G.emKS[ii] : 0;
    const sf_barrett EB = (emul || tens) ? loadBar(bar, prime) : sf_barrett{};
    const size_t trow = (size_t)ii << logn;
#pragma unroll
    for (int k = 0; k < NPAIR; ++k) {
        const uint32_t e = 2 * (threadIdx.x + k * NT);
        const size_t g = tileOff(k);
        ulonglong2 x;
        x.x = s[ldsSw(e)];
        x.y = s[ldsSw(e + 1)];
        if (fp) {  // every FP pass ends canonical: [0, q) as u64
            const double qd = (double)q, qi = qinvD[prime];
            double a0 = __longlong_as_double(x.x), a1 = __longlong_as_double(x.y);
            if (post) {  // stored as doubles: the fused conversion multiplies them as they are
                const double pd = G.postD[ii], pq = G.postQ[ii];
                x.x = __double_as_longlong(fpReduce(fpMulMod(a0, pd, pq, qd), qd, qi));
                x.y = __double_as_longlong(fpReduce(fpMulMod(a1, pd, pq, qd), qd, qi));
            } else {
                if (scale) {
                    a0 = fpMulMod(a0, ninvD[prime], ninvQ[prime], qd);
                    a1 = fpMulMod(a1, ninvD[prime], ninvQ[prime], qd);
                }
                x.x = d2u(fpReduce(a0, qd, qi));
                x.y = d2u(fpReduce(a1, qd, qi));
            }
        } else if (!FIRST) {  // finish the lazy ranges: forward [0,4q), inverse [0,2q) -> [0,q)
            if (scale) {
                x.x = sf_mul_shoup_lazy(x.x, ni, niS, q);
                x.y = sf_mul_shoup_lazy(x.y, ni, niS, q);
            } else {
                x.x = x.x >= 2 * q ? x.x - 2 * q : x.x;
                x.y = x.y >= 2 * q ? x.y - 2 * q : x.y;
            }
            x.x = x.x >= q ? x.x - q : x.x;
            x.y = x.y >= q ? x.y - q : x.y;
        }
        if (epi) {  // (the input row is read here: loaded with the tile it cost a wave per SIMD)
            ulonglong2 a = *reinterpret_cast<const ulonglong2*>(ein + g);
            if (emul) {
                const ulonglong2 m = *reinterpret_cast<const ulonglong2*>(emul + g);
                a.x = bmul(a.x, m.x, EB);
                a.y = bmul(a.y, m.y, EB);
            }
            if (emK) {
                a.x = sf_mul_shoup(a.x, emk, emkS, q);
                a.y = sf_mul_shoup(a.y, emk, emkS, q);
            }
            x.x = sf_mul_shoup(sf_sub(a.x, x.x, q), ek, ekS, q);
            x.y = sf_mul_shoup(sf_sub(a.y, x.y, q), ek, ekS, q);
            if ((G.addMask >> pp) & 1u) {
                const ulonglong2 o = *reinterpret_cast<const ulonglong2*>(out + g);
                x.x = sf_add(x.x, o.x, q);
                x.y = sf_add(x.y, o.y, q);
            }
            if (ead || tens) {
                ulonglong2 o;
                if (tens) {  // the tensor product's polynomial pp at (row ii, g)
                    const ulonglong2 a0 = *reinterpret_cast<const ulonglong2*>(G.tA0 + trow + g);
                    const ulonglong2 b0 = *reinterpret_cast<const ulonglong2*>(G.tB0 + trow + g);
                    if (pp == 0) {
                        o.x = bmul(a0.x, b0.x, EB);
                        o.y = bmul(a0.y, b0.y, EB);
                    } else {
                        const ulonglong2 a1 = *reinterpret_cast<const ulonglong2*>(G.tA1 + trow + g);
                        const ulonglong2 b1 = *reinterpret_cast<const ulonglong2*>(G.tB1 + trow + g);
                        Acc t{0, 0}, u{0, 0};
                        macc(t, a0.x, b1.x);
                        macc(t, a1.x, b0.x);
                        macc(u, a0.y, b1.y);
                        macc(u, a1.y, b0.y);
                        o.x = sf_reduce128_acc(t.lo, t.hi, &EB);
                        o.y = sf_reduce128_acc(u.lo, u.hi, &EB);
                    }
                } else {
                    o = *reinterpret_cast<const ulonglong2*>(ead + g);
                }
                x.x = sf_add(x.x, sf_mul_shoup(o.x, ek2, ek2S, q), q);
                x.y = sf_add(x.y, sf_mul_shoup(o.y, ek2, ek2S, q), q);
            }
        }
        *reinterpret_cast<ulonglong2*>(out + g) = x;
    }
    NTT_MARK(5);
#ifdef SFHE_NTT_TRACE
    if (threadIdx.x == 0) {
        auto& slot = g_nttTrace[(blockIdx.x + blockIdx.y * gridDim.x) % kTraceSlots][INV * 2 + COL];
        for (int i = 0; i < 6; ++i) atomicAdd(&slot[i], tacc[i]);
        atomicAdd(&slot[7], 1ull);
    }
#endif
}

// ModUp's conversion + forward COL pass for TG target rows per block
// (ModUpPlan, ring 2^16): the digit's source tiles are read once and feed
// all TG targets' conversion sums (k_ntt<..., CONV> reads them once per
// target: TG times the L2 traffic), then each target's tile runs the four COL
// rounds in LDS and is stored, as k_ntt's COL pass stores it (FP64 rows
// canonical, the integer row q_0 in the lazy forward range).  Grid row
// (p, g): digit p, targets g TG .. g TG + TG - 1 of its ell + K rows (the
// digit's own rows and rows past the end skipped).  Same signature as k_ntt
// (the merged-launch machinery), unused arguments ignored.
#ifndef SFHE_MODUP_TG
#define SFHE_MODUP_TG 4
#endif
constexpr int kModupTg = SFHE_MODUP_TG;
template <int TILE, int NG, int TG>
__global__ __launch_bounds__(TILE >> 2) void k_modup_col(const RowGroupSet<NG> GS, const sf_barrett* __restrict__ bar,
                                                         const u64* __restrict__ tw, const u64* __restrict__ twS,
                                                         const u64* __restrict__, const u64* __restrict__,
                                                         uint32_t logn, const double* __restrict__ twD,
                                                         const double* __restrict__ qinvD,
                                                         const double* __restrict__, const double* __restrict__,
                                                         int useFp, const double* __restrict__) {
    constexpr int LE = 2, NT = TILE >> LE, NPAIR = (1 << LE) / 2;
    __shared__ u64 s[TILE];
    __shared__ u64 tW[kNttColTw], tX[kNttColTw];
    const uint32_t n = 1u << logn;
    const uint32_t logR = logn - 8;  // (8: ring 2^16, checked on the host)
    uint32_t rid;
    const RowGroup& G = GS.a[argSel(GS, rid)];
    const uint32_t RG = (G.R + TG - 1) / TG;
    const uint32_t pp = rid / RG, g0 = (rid % RG) * TG;
    const uint32_t own0 = pp * G.alpha, own1 = min(own0 + G.alpha, G.skipEll);
    bool live[TG];  // (compile-time indexed: no scratch)
    bool any = false;
#pragma unroll
    for (int u = 0; u < TG; ++u) {
        const uint32_t ii = g0 + u;
        live[u] = ii < G.R && !(ii >= own0 && ii < own1);
        any = any || live[u];
    }
    if (!any) return;
    NttTile T;
    T.logn = logn;
    T.d = logR;
    T.logC = (uint32_t)__builtin_ctz(TILE) - logR;
    T.C = 1u << T.logC;
    const uint32_t tile = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    T.c0 = tile * T.C;
    T.r0 = 0;
    auto tileOff = [&](int k) -> size_t {
        const uint32_t e = 2 * (threadIdx.x + k * NT);
        return (size_t)(e >> T.logC) * 256 + T.c0 + (e & (T.C - 1));
    };
    const uint32_t ns = own1 - own0;
    const u64* yb = G.cy + (size_t)own0 * n;
    const bool big0 = G.cBig && pp == 0;
    // the targets' arithmetic: FP64 rows take the shared source pass; the
    // integer row (q_0, digits > 0) takes a pass of its own below
    uint32_t prime[TG];
    double qd[TG], qi[TG];
    bool fpT[TG];
    int nfp = 0;
#pragma unroll
    for (int u = 0; u < TG; ++u) {
        prime[u] = primeOf(G.pm, min(g0 + u, G.R - 1));
        const u64 q = bar[prime[u]].q;
        fpT[u] = useFp && q < kFpPrimeBound;
        qd[u] = (double)q;
        qi[u] = qinvD[prime[u]];
        nfp += live[u] && fpT[u];
    }
    double acc[TG][2 * NPAIR];
#pragma unroll
    for (int u = 0; u < TG; ++u)
#pragma unroll
        for (int w = 0; w < 2 * NPAIR; ++w) acc[u][w] = 0.0;
    if (nfp) {
        constexpr int GRP = 4;
        for (uint32_t s0 = 0; s0 < ns; s0 += GRP) {
            ulonglong2 v[GRP][NPAIR];
#pragma unroll
            for (int g = 0; g < GRP; ++g)
                if (s0 + g < ns)
#pragma unroll
                    for (int k = 0; k < NPAIR; ++k)
                        v[g][k] = *reinterpret_cast<const ulonglong2*>(yb + (size_t)(s0 + g) * n + tileOff(k));
#pragma unroll
            for (int g = 0; g < GRP; ++g) {
                const uint32_t sI = s0 + g;
                if (sI >= ns) break;
                const size_t mrow = (size_t)(own0 + sI) * G.cRows;
                const bool split = big0 && sI == 0;  // y < 2^60: y_lo + 2^30 y_hi
                double y[2 * NPAIR], yh[2 * NPAIR];
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {
                    if (split) {
                        y[2 * k] = u2d(v[g][k].x & 0x3fffffffull);
                        y[2 * k + 1] = u2d(v[g][k].y & 0x3fffffffull);
                        yh[2 * k] = u2d(v[g][k].x >> 30);
                        yh[2 * k + 1] = u2d(v[g][k].y >> 30);
                    } else {
                        y[2 * k] = __longlong_as_double(v[g][k].x);
                        y[2 * k + 1] = __longlong_as_double(v[g][k].y);
                    }
                }
#pragma unroll
                for (int u = 0; u < TG; ++u) {
                    if (!live[u] || !fpT[u]) continue;
                    const double md = G.cmD[mrow + g0 + u], mq = G.cmQ[mrow + g0 + u];
#pragma unroll
                    for (int w = 0; w < 2 * NPAIR; ++w) acc[u][w] += fpMulMod(y[w], md, mq, qd[u]);
                    if (split) {
                        const double hd = G.chD[g0 + u], hq = G.chQ[g0 + u];
#pragma unroll
                        for (int w = 0; w < 2 * NPAIR; ++w) acc[u][w] += fpMulMod(yh[w], hd, hq, qd[u]);
                    }
                }
            }
        }
    }
    constexpr int kColPer = (int)((kNttColTw + NT - 1) / NT);
    const uint32_t colTw = (1u << logR) - 1;
    bool first = true;
#pragma unroll
    for (int u = 0; u < TG; ++u) {
        if (!live[u]) continue;
        const uint32_t ii = g0 + u, pr = prime[u];
        const bool fp = fpT[u];
        const u64 q = bar[pr].q;
        ulonglong2 xr[NPAIR];
        if (fp) {
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {  // |acc| < 14 * 1.5 q < 2^46: exact
                xr[k].x = __double_as_longlong(fpReduce(acc[u][2 * k], qd[u], qi[u]));
                xr[k].y = __double_as_longlong(fpReduce(acc[u][2 * k + 1], qd[u], qi[u]));
            }
        } else {  // 128-bit sums of canonical residues
            const sf_barrett CB = loadBar(bar, pr);
            Acc a2[2 * NPAIR];
#pragma unroll
            for (int w = 0; w < 2 * NPAIR; ++w) a2[w] = Acc{0, 0};
            for (uint32_t sI = 0; sI < ns; ++sI) {
                const u64 m = G.cmI[(size_t)(own0 + sI) * G.cRows + ii];
                const bool raw = big0 && sI == 0;
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {
                    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(yb + (size_t)sI * n + tileOff(k));
                    macc(a2[2 * k], raw ? v.x : d2u(__longlong_as_double(v.x)), m);
                    macc(a2[2 * k + 1], raw ? v.y : d2u(__longlong_as_double(v.y)), m);
                }
            }
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {
                xr[k].x = sf_reduce128_acc(a2[2 * k].lo, a2[2 * k].hi, &CB);
                xr[k].y = sf_reduce128_acc(a2[2 * k + 1].lo, a2[2 * k + 1].hi, &CB);
            }
        }
        // the pass's twiddles for this prime, the tile -> LDS
        const u64* gwI = tw + (size_t)pr * n;
        const u64* gwD = reinterpret_cast<const u64*>(twD) + (size_t)pr * n;
        const u64* gx = twS + (size_t)pr * n;
        if (!first) __syncthreads();  // the previous target's readers are done with s / tW
        first = false;
#pragma unroll
        for (int c = 0; c < kColPer; ++c) {
            const uint32_t e = threadIdx.x + c * NT;
            if (e < colTw) {
                tW[e] = fp ? gwD[e + 1] : gwI[e + 1];
                if (!fp) tX[e] = gx[e + 1];
            }
        }
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) {
            const uint32_t e = 2 * (threadIdx.x + k * NT);
            s[ldsSw(e)] = xr[k].x;
            s[ldsSw(e + 1)] = xr[k].y;
        }
        __syncthreads();
        if (fp) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                nttRoundFP<false, true, 2, 2, TILE, false, 8>(reinterpret_cast<double*>(s), T, 0u, 2 * r, qd[u],
                                                              reinterpret_cast<const double*>(tW), qi[u]);
                __syncthreads();
            }
        } else {
            for (uint32_t r = 0; r < 4; ++r) {
                nttRoundDyn<false, true, LE, TILE>(2, s, T, 0u, LE * r, q, tW, tX);
                __syncthreads();
            }
        }
        u64* out = rowAt(G.dst, pp, ii);
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) {
            const uint32_t e = 2 * (threadIdx.x + k * NT);
            ulonglong2 x;
            x.x = s[ldsSw(e)];
            x.y = s[ldsSw(e + 1)];
            if (fp) {
                x.x = d2u(fpReduce(__longlong_as_double(x.x), qd[u], qi[u]));
                x.y = d2u(fpReduce(__longlong_as_double(x.y), qd[u], qi[u]));
            }
            *reinterpret_cast<ulonglong2*>(out + tileOff(k)) = x;
        }
    }
}

// Rings of at most one tile per row (n <= kNttTile = 2^11: the test
// rings the reference's k-way unit tests use, 2^10): the whole row in LDS, every
// stage in one block, exact radix-2 butterflies (the oracle's schedule, so
// canonical outputs), the same prologue (copy / pre / preK / lift) and
// epilogue (epi / emul / emK / addMask / eadd) as the two-pass kernel.  Not a
// performance path: one 256-thread block per row.
constexpr int kNttSmallThreads = 256;
template <bool INV>
__global__ __launch_bounds__(kNttSmallThreads) void k_ntt_small(const RowGroup G, const sf_barrett* __restrict__ bar,
                                                               const u64* __restrict__ tw, const u64* __restrict__ twS,
                                                               const u64* __restrict__ ninv,
                                                               const u64* __restrict__ ninvS, uint32_t logn) {
    __shared__ u64 s[kNttTile];
    const uint32_t n = 1u << logn;
    const uint32_t rid = blockIdx.y;
    const uint32_t pp = rid / G.R, ii = rid % G.R;
    if (G.skipEll && ii >= G.alpha * pp && ii < min(G.alpha * (pp + 1), G.skipEll)) return;
    const uint32_t prime = primeOf(G.pm, ii);
    const u64 q = bar[prime].q;
    const u64* in = rowAt(G.src, pp, ii);
    u64* cp = nullptr;
    if (G.copy.base)
        cp = G.copyByAlpha ? const_cast<u64*>(G.copy.base) + (ii / G.alpha) * G.copy.ps + ii * G.copy.is
                           : rowAt(G.copy, pp, ii);
    const u64* pre = G.pre.base ? rowAt(G.pre, pp, ii) : nullptr;
    const bool preK = G.preK != nullptr;
    const u64 pk = preK ? G.preK[ii] : 0, pkS = preK ? G.preKS[ii] : 0;
    const sf_barrett LB = (G.lift || pre) ? loadBar(bar, prime) : sf_barrett{};
    const u64 lsub = G.lift ? G.liftSub[ii] : 0;
    const u64 lhalf = G.lift ? (bar[G.liftPrime].q >> 1) : 0;
    for (uint32_t x = threadIdx.x; x < n; x += kNttSmallThreads) {
        u64 v = in[x];
        if (cp) cp[x] = v;
        if (pre) v = bmul(v, pre[x], LB);
        if (preK) v = sf_mul_shoup(v, pk, pkS, q);
        if (G.lift) {
            u64 r = sf_reduce128(v, 0, &LB);
            v = v > lhalf ? sf_sub(r, lsub, q) : r;
        }
        s[x] = v;
    }
    __syncthreads();
    const u64* w = tw + (size_t)prime * n;
    const u64* wS = twS + (size_t)prime * n;
    for (uint32_t st = 0; st < logn; ++st) {
        // forward: m = 2^st groups of span 2t; inverse: the same stages reversed
        const uint32_t m = INV ? (n >> (st + 1)) : (1u << st);
        const uint32_t t = (n >> 1) / m;
        for (uint32_t b = threadIdx.x; b < n / 2; b += kNttSmallThreads) {
            const uint32_t i = b / t, j = b % t, x = 2 * i * t + j;
            const u64 S = w[m + i], Sp = wS[m + i];
            const u64 U = s[x], V = s[x + t];
            if (INV) {
                s[x] = sf_add(U, V, q);
                s[x + t] = sf_mul_shoup(sf_sub(U, V, q), S, Sp, q);
            } else {
                const u64 VW = sf_mul_shoup(V, S, Sp, q);
                s[x] = sf_add(U, VW, q);
                s[x + t] = sf_sub(U, VW, q);
            }
        }
        __syncthreads();
    }
    const bool epi = G.epi != 0;
    u64* out = epi ? rowAt(G.eout, pp, ii) : rowAt(G.dst, pp, ii);
    const u64* ein = epi ? rowAt(G.ein, pp, ii) : nullptr;
    const u64 ek = epi ? G.k[ii] : 0, ekS = epi ? G.kS[ii] : 0;
    const u64* ead = epi && G.eadd.base ? rowAt(G.eadd, pp, ii) : nullptr;
    const u64 ek2 = ead ? G.k2[ii] : 0, ek2S = ead ? G.k2S[ii] : 0;
    const u64* emul = epi && G.emul.base ? rowAt(G.emul, pp, ii) : nullptr;
    const bool emK = epi && G.emK;
    const u64 emk = emK ? G.emK[ii] : 0, emkS = emK ? G.emKS[ii] : 0;
    const sf_barrett EB = emul ? loadBar(bar, prime) : sf_barrett{};
    for (uint32_t x = threadIdx.x; x < n; x += kNttSmallThreads) {
        u64 v = s[x];
        if (INV) v = sf_mul_shoup(v, ninv[prime], ninvS[prime], q);
        if (epi) {
            u64 a = ein[x];
            if (emul) a = bmul(a, emul[x], EB);
            if (emK) a = sf_mul_shoup(a, emk, emkS, q);
            v = sf_mul_shoup(sf_sub(a, v, q), ek, ekS, q);
            if ((G.addMask >> pp) & 1u) v = sf_add(v, out[x], q);
            if (ead) v = sf_add(v, sf_mul_shoup(ead[x], ek2, ek2S, q), q);
        }
        out[x] = v;
    }
}

// ============================================================================
// elementwise kernels: one thread per pair of coefficients (16 B per lane)

enum EwOp { EW_ADD, EW_SUB, EW_NEG, EW_MUL, EW_MULADD, EW_MULC, EW_ADDC };

// ---- ModUp's last NTT pass fused with the key inner product ----------------
// (sfp_modup_inner).  Block (tile, t) owns row-tile `tile` of extended-basis
// limb t.  For every digit j it takes that limb's canonical evaluation-domain
// tile -- the forward ROW pass of the COL-pass output in ext_j, or the input
// row itself where t is one of digit j's own limbs -- multiplies it by digit
// j's two key rows and accumulates 128-bit sums; after the last digit the
// sums (+ the relinearisation fold, + the previous accumulator) are reduced
// into acc rows t.  The same integers as the ROW pass writing ext followed by
// k_ks_inner, without the ext round trip through HBM and the extra launch.
struct KsArgs {
    const u64* in;        // ell rows, evaluation domain (the digits' own limbs)
    const u64* inMul;     // non-null: the own limbs are in (.) inMul (a relinearised tensor's d2 = a1 b1)
    const u64* ext;       // beta blocks of ell+K rows: COL-pass output of the other limbs
    long long extStride;  // words between digit blocks
    const u64* key;       // beta digits of [b rows][a rows], keyRows rows each
    uint32_t keyRows, keyQ;  // ext limb t uses key row t < ell ? t : keyQ + (t - ell)
    u64* acc0;
    u64* acc1;
    const u64* fold0;  // t == ell - 1: + foldK * fold_p (sfp_ks_inner_fold)
    const u64* fold1;
    u64 foldK;
    // non-null: the fold rows are the tensor's d0 = a0 b0, d1 = a0 b1 + a1 b0
    // at row ell - 1, formed here (fold0 / fold1 unused)
    const u64 *fa0, *fa1, *fb0, *fb1;
    uint32_t ell, Lq, alpha, beta;
    int accum;  // acc += the inner product
    // rows t >= invFrom (the P limbs, and for a ModDown fused with its rescale
    // the dropped q limb too) leave after the first pass of ModDown's inverse
    // NTT (its ROW pass), which the ModDown then skips; ~0u: none
    uint32_t invFrom;
    const u64 *itw, *itwS;
    const double* itwD;
};

template <int LE, int TILE, int NG = 1>
__global__ __launch_bounds__(TILE >> LE) void k_ntt_ks(const ArgSet<KsArgs, NG> AS, const sf_barrett* __restrict__ bar,
                                                     const u64* __restrict__ tw, const u64* __restrict__ twS,
                                                     uint32_t logn, const double* __restrict__ twD,
                                                     const double* __restrict__ qinvD, int useFp,
                                                     const double* __restrict__ rowD) {
    __shared__ u64 s[2 * TILE];  // the second tile: acc1's inverse ROW pass (same rounds as acc0's)
    constexpr int NT = TILE >> LE;       // threads
    constexpr int NPAIR = (1 << LE) / 2;  // 16-byte pairs per thread
    const uint32_t n = 1u << logn;
    const uint32_t logR = logn - 8;
    uint32_t t;
    const KsArgs& A = AS.a[argSel(AS, t)];
    const uint32_t prime = t < A.ell ? t : A.Lq + (t - A.ell);
    const sf_barrett B = loadBar(bar, prime);
    const u64 q = B.q;
    const bool fp = useFp && q < kFpPrimeBound;
    NttTile T;
    T.logn = logn;
    T.d = 8u;
    T.logC = 0;
    T.C = 1;
    const uint32_t tile = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    T.c0 = 0;
    T.r0 = tile * (TILE / 256);
    const uint32_t S0 = logR;
    const u64* gw = fp ? reinterpret_cast<const u64*>(twD) + (size_t)prime * n : tw + (size_t)prime * n;
    const u64* gx = twS + (size_t)prime * n;
    constexpr bool kPfBuild = LE == 2;
    constexpr int kPfRounds = 4;
#ifndef SFHE_KS_PW_LOOP
#define SFHE_KS_PW_LOOP 1
#endif
    // the ROW rounds' FP64 twiddles, 12 per thread: loaded once per digit
    // (SFHE_KS_PW_LOOP, keeping them live across the digits costs a wave per
    // SIMD) or once per block
    // (the full table, not rowTwIssue's factors: the products' registers cost
    // this kernel a wave per SIMD, and its twiddle bytes are < 10 % of its
    // key and digit traffic)
    auto loadPW = [&](double* PW) {
        if constexpr (kPfBuild) {
            const double* gd = reinterpret_cast<const double*>(gw);
#pragma unroll
            for (int r = 0; r < kPfRounds; ++r) {
                const uint32_t k0 = 2 * r, logh = 8 - k0 - 2;
                const uint32_t lo = threadIdx.x & ((1u << logh) - 1);
                const uint32_t rest = threadIdx.x >> logh;
                const uint32_t hi = rest & ((1u << k0) - 1);
                const uint32_t st = rest >> k0;
                const uint32_t x0 = nttGlobal<false>(T, st, hi * (256u >> k0) + lo);
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    const uint32_t tb = twIndex<false>(T, S0, k0 + tt, x0);
#pragma unroll
                    for (int qd = 0; qd < (1 << tt); ++qd) PW[3 * r + (1 << tt) - 1 + qd] = gd[tb + qd];
                }
            }
        }
    };
    double PW[kPfBuild ? kPfRounds * 3 : 1];
    if (!SFHE_KS_PW_LOOP && fp) loadPW(PW);
    const double qd = (double)q, qi = qinvD[prime];
    const uint32_t kr = t < A.ell ? t : A.keyQ + (t - A.ell);
    const size_t rowOff = (size_t)T.r0 * 256;
    const bool inv = t >= A.invFrom;
    const u64* iw = fp ? reinterpret_cast<const u64*>(A.itwD) + (size_t)prime * n : A.itw + (size_t)prime * n;
    const u64* ix = A.itwS + (size_t)prime * n;
    // Each digit's key rows are issued before the ROW rounds that precede
    // their use (loads in flight hide their latency at this occupancy).
    u64* o0 = A.acc0 + (size_t)t * n + rowOff;
    u64* o1 = A.acc1 + (size_t)t * n + rowOff;
    // The digits' products: FP64 rows (every row but q_0 at the metric's
    // parameters) accumulate exact residues of each product (fpMulMod: an
    // integer-valued double congruent to v * key, |r| < 2^45, so the few
    // digits' and the fold's terms sum exactly below 2^52); the integer row
    // accumulates 128-bit sums.  Either way the stored value is the canonical
    // residue of the same sum (bit-identical outputs).
    auto body = [&](auto fpTag) {
        constexpr bool FP = decltype(fpTag)::value;
        using AccT = std::conditional_t<FP, double, Acc>;
        AccT a0[2 * NPAIR], a1[2 * NPAIR];
#pragma unroll
        for (int w = 0; w < 2 * NPAIR; ++w) {
            if constexpr (FP) a0[w] = a1[w] = 0.0;
            else a0[w] = a1[w] = Acc{0, 0};
        }
        // (a * b mod q for canonical u64 operands, as the accumulator's term)
        auto term = [&](AccT& acc, auto x, u64 w) {
            if constexpr (FP) {
                const double wd = u2d(w);
                double y;
                if constexpr (std::is_same_v<decltype(x), u64>) y = u2d(x);
                else y = x;
                acc += fpMulMod(y, wd, wd * qi, qd);
            } else {
                macc(acc, (u64)x, w);
            }
        };
        for (uint32_t j = 0; j < A.beta; ++j) {
            const bool own = t < A.ell && t >= j * A.alpha && t < min((j + 1) * A.alpha, A.ell);
            std::conditional_t<FP, double, u64> v[2 * NPAIR];
            const u64* kb = A.key + (size_t)j * 2 * A.keyRows * n + (size_t)kr * n + rowOff;
            const u64* ka = kb + (size_t)A.keyRows * n;
            ulonglong2 kb2[NPAIR], ka2[NPAIR];
            if (own) {
                const u64* src = A.in + (size_t)t * n + rowOff;
                const u64* mul = A.inMul ? A.inMul + (size_t)t * n + rowOff : nullptr;
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {
                    const uint32_t e = 2 * (threadIdx.x + k * NT);
                    ulonglong2 x = *reinterpret_cast<const ulonglong2*>(src + e);
                    if (mul) {
                        const ulonglong2 m = *reinterpret_cast<const ulonglong2*>(mul + e);
                        x.x = bmul(x.x, m.x, B);
                        x.y = bmul(x.y, m.y, B);
                    }
                    if constexpr (FP) {
                        v[2 * k] = u2d(x.x);
                        v[2 * k + 1] = u2d(x.y);
                    } else {
                        v[2 * k] = x.x;
                        v[2 * k + 1] = x.y;
                    }
                }
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {
                    const uint32_t e = 2 * (threadIdx.x + k * NT);
                    kb2[k] = *reinterpret_cast<const ulonglong2*>(kb + e);
                    ka2[k] = *reinterpret_cast<const ulonglong2*>(ka + e);
                }
            } else {
                const u64* src = A.ext + j * A.extStride + (size_t)t * n + rowOff;
                ulonglong2 xs[NPAIR];
#pragma unroll
                for (int k = 0; k < NPAIR; ++k)
                    xs[k] = *reinterpret_cast<const ulonglong2*>(src + 2 * (threadIdx.x + k * NT));
                if constexpr (FP && SFHE_KS_PW_LOOP) loadPW(PW);
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {  // in flight during the ROW rounds
                    const uint32_t e = 2 * (threadIdx.x + k * NT);
                    kb2[k] = *reinterpret_cast<const ulonglong2*>(kb + e);
                    ka2[k] = *reinterpret_cast<const ulonglong2*>(ka + e);
                }
                __syncthreads();  // the previous digit's readers are done with s
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {
                    const uint32_t e = 2 * (threadIdx.x + k * NT);
                    const ulonglong2 x = xs[k];
                    if constexpr (FP) {
                        s[ldsSw(e)] = __double_as_longlong(u2d(x.x));
                        s[ldsSw(e + 1)] = __double_as_longlong(u2d(x.y));
                    } else {
                        s[ldsSw(e)] = x.x;
                        s[ldsSw(e + 1)] = x.y;
                    }
                }
                __syncthreads();
                bool done = false;
                if constexpr (kPfBuild && FP) {
#pragma unroll
                    for (int r = 0; r < kPfRounds; ++r) {
                        nttRoundFP<false, false, 2, 2, TILE, true, 8>(reinterpret_cast<double*>(s), T, S0, 2 * r,
                                                                      qd, nullptr, qi, PW + 3 * r);
                        __syncthreads();
                    }
                    done = true;
                }
                if (!done) {
                    const uint32_t nr = (8 + LE - 1) / LE;
                    for (uint32_t r = 0; r < nr; ++r) {
                        const uint32_t k0 = LE * r;
                        const int b = (int)min((uint32_t)LE, 8u - k0);
                        if constexpr (FP)
                            nttRoundDynFP<false, false, LE, TILE>(b, reinterpret_cast<double*>(s), T, S0, k0, qd,
                                                                  reinterpret_cast<const double*>(gw), qi);
                        else
                            nttRoundDyn<false, false, LE, TILE>(b, s, T, S0, k0, q, gw, gx);
                        __syncthreads();
                    }
                }
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {
                    const uint32_t e = 2 * (threadIdx.x + k * NT);
                    u64 x0 = s[ldsSw(e)], x1 = s[ldsSw(e + 1)];
                    if constexpr (FP) {  // integer-valued doubles in the rounds' range: fpMulMod takes them as they are
                        v[2 * k] = __longlong_as_double(x0);
                        v[2 * k + 1] = __longlong_as_double(x1);
                    } else {  // forward lazy range [0, 4q) -> [0, q)
                        x0 = x0 >= 2 * q ? x0 - 2 * q : x0;
                        x1 = x1 >= 2 * q ? x1 - 2 * q : x1;
                        x0 = x0 >= q ? x0 - q : x0;
                        x1 = x1 >= q ? x1 - q : x1;
                        v[2 * k] = x0;
                        v[2 * k + 1] = x1;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {
                const ulonglong2 b2 = kb2[k];
                const ulonglong2 a2 = ka2[k];
                term(a0[2 * k], v[2 * k], b2.x);
                term(a0[2 * k + 1], v[2 * k + 1], b2.y);
                term(a1[2 * k], v[2 * k], a2.x);
                term(a1[2 * k + 1], v[2 * k + 1], a2.y);
            }
        }
        // the previous accumulator, loaded after the digits (holding it in
        // registers through them costs a wave per SIMD)
        ulonglong2 prev[2][NPAIR];
        if (A.accum) {
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {
                const uint32_t e = 2 * (threadIdx.x + k * NT);
                prev[0][k] = *reinterpret_cast<const ulonglong2*>(o0 + e);
                prev[1][k] = *reinterpret_cast<const ulonglong2*>(o1 + e);
            }
        }
        const bool fold = (A.fold0 || A.fa0) && t == A.ell - 1;
        if (inv) __syncthreads();  // the last digit's readers are done with s
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) {
            const uint32_t e = 2 * (threadIdx.x + k * NT);
            if (fold) {  // + P * d_l (sfp_ks_inner_fold)
                if (A.fa0) {  // d0 = a0 b0, d1 = a0 b1 + a1 b0 at row l (canonical, as k_tensor writes them)
                    const size_t ro = (size_t)t * n + rowOff + e;
                    const ulonglong2 x0 = *reinterpret_cast<const ulonglong2*>(A.fa0 + ro);
                    const ulonglong2 x1 = *reinterpret_cast<const ulonglong2*>(A.fa1 + ro);
                    const ulonglong2 y0 = *reinterpret_cast<const ulonglong2*>(A.fb0 + ro);
                    const ulonglong2 y1 = *reinterpret_cast<const ulonglong2*>(A.fb1 + ro);
                    if constexpr (FP) {
                        const double fk = u2d(A.foldK), fkq = fk * qi;
                        const double qx0 = u2d(x0.x), qy0 = u2d(x0.y), qx1 = u2d(x1.x), qy1 = u2d(x1.y);
                        const double b0x = u2d(y0.x), b0y = u2d(y0.y), b1x = u2d(y1.x), b1y = u2d(y1.y);
                        const double f0x = fpMulMod(qx0, b0x, b0x * qi, qd), f0y = fpMulMod(qy0, b0y, b0y * qi, qd);
                        const double f1x = fpMulMod(qx0, b1x, b1x * qi, qd) + fpMulMod(qx1, b0x, b0x * qi, qd);
                        const double f1y = fpMulMod(qy0, b1y, b1y * qi, qd) + fpMulMod(qy1, b0y, b0y * qi, qd);
                        a0[2 * k] += fpMulMod(f0x, fk, fkq, qd);
                        a0[2 * k + 1] += fpMulMod(f0y, fk, fkq, qd);
                        a1[2 * k] += fpMulMod(f1x, fk, fkq, qd);
                        a1[2 * k + 1] += fpMulMod(f1y, fk, fkq, qd);
                    } else {
                        Acc tt{0, 0}, uu{0, 0};
                        macc(tt, x0.x, y1.x);
                        macc(tt, x1.x, y0.x);
                        macc(uu, x0.y, y1.y);
                        macc(uu, x1.y, y0.y);
                        macc(a0[2 * k], bmul(x0.x, y0.x, B), A.foldK);
                        macc(a0[2 * k + 1], bmul(x0.y, y0.y, B), A.foldK);
                        macc(a1[2 * k], sf_reduce128_acc(tt.lo, tt.hi, &B), A.foldK);
                        macc(a1[2 * k + 1], sf_reduce128_acc(uu.lo, uu.hi, &B), A.foldK);
                    }
                } else {
                    const ulonglong2 f0 = *reinterpret_cast<const ulonglong2*>(A.fold0 + (size_t)t * n + rowOff + e);
                    const ulonglong2 f1 = *reinterpret_cast<const ulonglong2*>(A.fold1 + (size_t)t * n + rowOff + e);
                    term(a0[2 * k], f0.x, A.foldK);
                    term(a0[2 * k + 1], f0.y, A.foldK);
                    term(a1[2 * k], f1.x, A.foldK);
                    term(a1[2 * k + 1], f1.y, A.foldK);
                }
            }
            if constexpr (FP) {
                double r[4] = {a0[2 * k], a0[2 * k + 1], a1[2 * k], a1[2 * k + 1]};
                if (A.accum) {
                    r[0] += u2d(prev[0][k].x);
                    r[1] += u2d(prev[0][k].y);
                    r[2] += u2d(prev[1][k].x);
                    r[3] += u2d(prev[1][k].y);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) r[u] = fpReduce(r[u], qd, qi);
                if (!inv) {
                    *reinterpret_cast<ulonglong2*>(o0 + e) = make_ulonglong2(d2u(r[0]), d2u(r[1]));
                    *reinterpret_cast<ulonglong2*>(o1 + e) = make_ulonglong2(d2u(r[2]), d2u(r[3]));
                } else {
                    s[ldsSw(e)] = __double_as_longlong(r[0]);
                    s[ldsSw(e + 1)] = __double_as_longlong(r[1]);
                    s[TILE + ldsSw(e)] = __double_as_longlong(r[2]);
                    s[TILE + ldsSw(e + 1)] = __double_as_longlong(r[3]);
                }
            } else {
                ulonglong2 r0, r1;
                r0.x = sf_reduce128_acc(a0[2 * k].lo, a0[2 * k].hi, &B);
                r0.y = sf_reduce128_acc(a0[2 * k + 1].lo, a0[2 * k + 1].hi, &B);
                r1.x = sf_reduce128_acc(a1[2 * k].lo, a1[2 * k].hi, &B);
                r1.y = sf_reduce128_acc(a1[2 * k + 1].lo, a1[2 * k + 1].hi, &B);
                if (A.accum) {
                    const ulonglong2 p0 = prev[0][k], p1 = prev[1][k];
                    r0.x = sf_add(r0.x, p0.x, q);
                    r0.y = sf_add(r0.y, p0.y, q);
                    r1.x = sf_add(r1.x, p1.x, q);
                    r1.y = sf_add(r1.y, p1.y, q);
                }
                if (!inv) {
                    *reinterpret_cast<ulonglong2*>(o0 + e) = r0;
                    *reinterpret_cast<ulonglong2*>(o1 + e) = r1;
                } else {
                    s[ldsSw(e)] = r0.x;
                    s[ldsSw(e + 1)] = r0.y;
                    s[TILE + ldsSw(e)] = r1.x;
                    s[TILE + ldsSw(e + 1)] = r1.y;
                }
            }
        }
    };
    if (fp)
        body(std::true_type{});
    else
        body(std::false_type{});
    if (!inv) return;
    // ModDown's inverse ROW pass on both accumulators' tiles, round by round
    // (as k_ntt's first inverse pass: FP64 rows leave canonical, integer rows
    // in [0, 2q)); its twiddles are loaded here, after the digits
    double PIW[kPfBuild ? kPfRounds * 3 : 1];
    if constexpr (kPfBuild) {
        if (fp && inv) {
            const double* gd = reinterpret_cast<const double*>(iw);
#pragma unroll
            for (int r = 0; r < kPfRounds; ++r) {
                const uint32_t k0 = 2 * r, logh = 8 - k0 - 2;
                const uint32_t lo = threadIdx.x & ((1u << logh) - 1);
                const uint32_t rest = threadIdx.x >> logh;
                const uint32_t hi = rest & ((1u << k0) - 1);
                const uint32_t st = rest >> k0;
                const uint32_t x0 = nttGlobal<false>(T, st, hi * (256u >> k0) + lo);
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    const uint32_t tb = twIndex<false>(T, S0, k0 + tt, x0);
#pragma unroll
                    for (int qd2 = 0; qd2 < (1 << tt); ++qd2) PIW[3 * r + (1 << tt) - 1 + qd2] = gd[tb + qd2];
                }
            }
        }
    }
    __syncthreads();
    bool done = false;
    if constexpr (kPfBuild) {
        if (fp) {
#pragma unroll
            for (int ri = 0; ri < kPfRounds; ++ri) {
                const int r = kPfRounds - 1 - ri;
                nttRoundFP<true, false, 2, 2, TILE, true, 8>(reinterpret_cast<double*>(s), T, S0, 2 * r, qd, nullptr,
                                                             qi, PIW + 3 * r);
                nttRoundFP<true, false, 2, 2, TILE, true, 8>(reinterpret_cast<double*>(s + TILE), T, S0, 2 * r, qd,
                                                             nullptr, qi, PIW + 3 * r);
                __syncthreads();
            }
            done = true;
        }
    }
    if (!done) {
        const uint32_t nr = (8 + LE - 1) / LE;
        for (uint32_t ri = 0; ri < nr; ++ri) {
            const uint32_t rr = nr - 1 - ri;
            const uint32_t k0 = LE * rr;
            const int b = (int)min((uint32_t)LE, 8u - k0);
            for (int p = 0; p < 2; ++p) {
                if (fp)
                    nttRoundDynFP<true, false, LE, TILE>(b, reinterpret_cast<double*>(s + p * TILE), T, S0, k0, qd,
                                                         reinterpret_cast<const double*>(iw), qi);
                else
                    nttRoundDyn<true, false, LE, TILE>(b, s + p * TILE, T, S0, k0, q, iw, ix);
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        u64* o = p ? o1 : o0;
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) {
            const uint32_t e = 2 * (threadIdx.x + k * NT);
            ulonglong2 x;
            x.x = s[p * TILE + ldsSw(e)];
            x.y = s[p * TILE + ldsSw(e + 1)];
            if (fp) {
                x.x = d2u(fpReduce(__longlong_as_double(x.x), qd, qi));
                x.y = d2u(fpReduce(__longlong_as_double(x.y), qd, qi));
            }
            *reinterpret_cast<ulonglong2*>(o + e) = x;
        }
    }
}

struct ConstArgs {
    u64 k[SFP_MAX_LIMBS];
};

// Grid-stride kernels in arg-set form: set blockIdx.y of NG (a stacked pair
// of launches runs both sets, grid.y = 2; each set loops over its own rows).
struct EwArgs {
    u64* out;
    const u64 *a, *b, *c;
    sfp_limbs m;
    ConstArgs k;
};
template <int OP, int NG = 1>
__global__ __launch_bounds__(kThreads) void k_ew(const ArgSet<EwArgs, NG> S, const sf_barrett* __restrict__ bar,
                                                 uint32_t logn) {
    const EwArgs& A = S.a[NG > 1 ? blockIdx.y : 0];
    u64* __restrict__ out = A.out;
    const u64* __restrict__ a = A.a;
    const u64* __restrict__ b = A.b;
    const u64* __restrict__ c = A.c;
    const sfp_limbs m = A.m;
    const ConstArgs& k = A.k;
    const size_t pairs = ((size_t)m.count << logn) >> 1;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < pairs;
         i += (size_t)gridDim.x * kThreads) {
        const uint32_t limb = (uint32_t)((2 * i) >> logn);
        const sf_barrett B = loadBar(bar, primeOf(m, limb));
        const u64 q = B.q;
        ulonglong2 x = reinterpret_cast<const ulonglong2*>(a)[i];
        ulonglong2 r;
        if (OP == EW_ADD || OP == EW_SUB || OP == EW_MUL || OP == EW_MULADD) {
            ulonglong2 y = reinterpret_cast<const ulonglong2*>(b)[i];
            if (OP == EW_ADD) {
                r.x = sf_add(x.x, y.x, q);
                r.y = sf_add(x.y, y.y, q);
            } else if (OP == EW_SUB) {
                r.x = sf_sub(x.x, y.x, q);
                r.y = sf_sub(x.y, y.y, q);
            } else {
                r.x = bmul(x.x, y.x, B);
                r.y = bmul(x.y, y.y, B);
                if (OP == EW_MULADD) {
                    ulonglong2 z = reinterpret_cast<const ulonglong2*>(c)[i];
                    r.x = sf_add(r.x, z.x, q);
                    r.y = sf_add(r.y, z.y, q);
                }
            }
        } else if (OP == EW_NEG) {
            r.x = sf_neg(x.x, q);
            r.y = sf_neg(x.y, q);
        } else if (OP == EW_MULC) {
            r.x = bmul(x.x, k.k[limb], B);
            r.y = bmul(x.y, k.k[limb], B);
        } else {  // EW_ADDC
            r.x = sf_add(x.x, k.k[limb], q);
            r.y = sf_add(x.y, k.k[limb], q);
        }
        reinterpret_cast<ulonglong2*>(out)[i] = r;
    }
}

__global__ __launch_bounds__(kThreads) void k_tensor(u64* __restrict__ d0, u64* __restrict__ d1,
                                                     u64* __restrict__ d2, const u64* __restrict__ a0,
                                                     const u64* __restrict__ a1, const u64* __restrict__ b0,
                                                     const u64* __restrict__ b1, sfp_limbs m,
                                                     const sf_barrett* __restrict__ bar, uint32_t logn) {
    // two coefficients per thread (16-byte loads and stores)
    const size_t pairs = ((size_t)m.count << logn) >> 1;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < pairs;
         i += (size_t)gridDim.x * kThreads) {
        const sf_barrett B = loadBar(bar, primeOf(m, (uint32_t)((2 * i) >> logn)));
        const ulonglong2 x0 = reinterpret_cast<const ulonglong2*>(a0)[i];
        const ulonglong2 x1 = reinterpret_cast<const ulonglong2*>(a1)[i];
        const ulonglong2 y0 = reinterpret_cast<const ulonglong2*>(b0)[i];
        const ulonglong2 y1 = reinterpret_cast<const ulonglong2*>(b1)[i];
        Acc t{0, 0}, u{0, 0};
        macc(t, x0.x, y1.x);
        macc(t, x1.x, y0.x);
        macc(u, x0.y, y1.y);
        macc(u, x1.y, y0.y);
        ulonglong2 r0, r1, r2;
        r0.x = bmul(x0.x, y0.x, B);
        r0.y = bmul(x0.y, y0.y, B);
        r1.x = sf_reduce128_acc(t.lo, t.hi, &B);
        r1.y = sf_reduce128_acc(u.lo, u.hi, &B);
        r2.x = bmul(x1.x, y1.x, B);
        r2.y = bmul(x1.y, y1.y, B);
        reinterpret_cast<ulonglong2*>(d0)[i] = r0;
        reinterpret_cast<ulonglong2*>(d1)[i] = r1;
        reinterpret_cast<ulonglong2*>(d2)[i] = r2;
    }
}

struct PtrList {
    const u64* p[SFP_MAX_WSUM];
};
struct PtrList2 {
    const u64* a[SFP_MAX_WSUM];
    const u64* b[SFP_MAX_WSUM];
};

// out = sum_j ins[j] * k[j][limb]   (k: device array nin x count)
struct WsumArgs {
    u64* out;
    PtrList ins;
    const u64* k;
    uint32_t nin;
    sfp_limbs m;
};
template <int NG = 1>
__global__ __launch_bounds__(kThreads) void k_lin_wsum(const ArgSet<WsumArgs, NG> S, const sf_barrett* __restrict__ bar,
                                                       uint32_t logn) {
    const WsumArgs& A = S.a[NG > 1 ? blockIdx.y : 0];
    u64* __restrict__ out = A.out;
    const PtrList& ins = A.ins;
    const u64* __restrict__ k = A.k;
    const uint32_t nin = A.nin;
    const sfp_limbs m = A.m;
    const size_t total = (size_t)m.count << logn;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < total;
         i += (size_t)gridDim.x * kThreads) {
        const uint32_t limb = (uint32_t)(i >> logn);
        const sf_barrett B = loadBar(bar, primeOf(m, limb));
        Acc acc{0, 0};
        for (uint32_t j = 0; j < nin; ++j) macc(acc, ins.p[j][i], k[(size_t)j * m.count + limb]);
        out[i] = sf_reduce128_acc(acc.lo, acc.hi, &B);
    }
}

// Multi-output weighted sum: grid (coefficient blocks, limb, chunk of
// kWsumChunk outputs).  Each thread streams the nin inputs of its coefficient
// once per chunk and keeps 2 x kWsumChunk 128-bit accumulators; the chunk's
// weights for this limb sit in LDS.
constexpr int kWsumChunk = 8;
__global__ __launch_bounds__(kThreads) void k_lin_wsum_multi(u64* __restrict__ out, size_t outStride,
                                                             size_t polyStride, PtrList2 ins,
                                                             const u64* __restrict__ k, uint32_t nin,
                                                             uint32_t nout, sfp_limbs m,
                                                             const sf_barrett* __restrict__ bar,
                                                             uint32_t logn, const double* __restrict__ qinvD,
                                                             int useFp) {
    __shared__ u64 sk[kWsumChunk * SFP_MAX_WSUM];
    // blockIdx.x -> (coefficient block, output chunk): every chunk re-streams
    // the nin inputs of its coefficients, so the chunks of one coefficient
    // block go to the same XCD (block id = XCD mod 8), 8 ids apart in dispatch
    // order, and their input reads meet in that XCD's L2
    const uint32_t chunks = (nout + kWsumChunk - 1) / kWsumChunk;
    const uint32_t cbs = gridDim.x / chunks;
    uint32_t cb, chunk;
    if ((cbs & 7) == 0) {
        const uint32_t r = blockIdx.x >> 3;
        chunk = r % chunks;
        cb = (r / chunks) * 8 + (blockIdx.x & 7);
    } else {
        chunk = blockIdx.x % chunks;
        cb = blockIdx.x / chunks;
    }
    const uint32_t limb = blockIdx.y;
    const uint32_t o0 = chunk * kWsumChunk;
    const uint32_t oc = min((uint32_t)kWsumChunk, nout - o0);
    // FP64 rows also stage each weight as (w, w/q) doubles: the product loop
    // then neither converts nor rescales a weight per coefficient
    __shared__ double skD[kWsumChunk * SFP_MAX_WSUM], skQ[kWsumChunk * SFP_MAX_WSUM];
    const uint32_t prime = primeOf(m, limb);
    const u64 qq = bar[prime].q;
    const bool fpRow = useFp && qq < kFpPrimeBound;  // uniform per block
    const double qi = fpRow ? qinvD[prime] : 0.0;
    for (uint32_t e = threadIdx.x; e < oc * nin; e += kThreads) {
        const uint32_t o = e / nin, j = e % nin;
        const u64 w = k[((size_t)(o0 + o) * nin + j) * m.count + limb];
        sk[o * SFP_MAX_WSUM + j] = w;
        if (fpRow) {
            skD[o * SFP_MAX_WSUM + j] = (double)w;
            skQ[o * SFP_MAX_WSUM + j] = (double)w * qi;
        }
    }
    __syncthreads();
    const uint32_t n = 1u << logn;
    const uint32_t x = cb * kThreads + threadIdx.x;
    if (x >= n) return;
    const size_t off = ((size_t)limb << logn) + x;
    if (fpRow) {  // FP64 products (fpMulMod), exact
        const double qd = (double)qq;
        double f0[kWsumChunk], f1[kWsumChunk];
#pragma unroll
        for (int o = 0; o < kWsumChunk; ++o) f0[o] = f1[o] = 0.0;
        for (uint32_t j = 0; j < nin; ++j) {  // |sum| < nin * 2q < 2^50
            const double v0 = (double)ins.a[j][off], v1 = (double)ins.b[j][off];
#pragma unroll
            for (int o = 0; o < kWsumChunk; ++o) {
                if ((uint32_t)o < oc) {
                    const double w = skD[o * SFP_MAX_WSUM + j], wq = skQ[o * SFP_MAX_WSUM + j];
                    f0[o] += fpMulMod(v0, w, wq, qd);
                    f1[o] += fpMulMod(v1, w, wq, qd);
                }
            }
        }
#pragma unroll
        for (int o = 0; o < kWsumChunk; ++o) {
            if ((uint32_t)o < oc) {
                u64* dst = out + (size_t)(o0 + o) * outStride + off;
                dst[0] = d2u(fpReduce(f0[o], qd, qi));
                dst[polyStride] = d2u(fpReduce(f1[o], qd, qi));
            }
        }
        return;
    }
    Acc a0[kWsumChunk], a1[kWsumChunk];
#pragma unroll
    for (int o = 0; o < kWsumChunk; ++o) a0[o] = a1[o] = Acc{0, 0};
    for (uint32_t j = 0; j < nin; ++j) {
        const u64 v0 = ins.a[j][off], v1 = ins.b[j][off];
#pragma unroll
        for (int o = 0; o < kWsumChunk; ++o) {
            if ((uint32_t)o < oc) {
                const u64 w = sk[o * SFP_MAX_WSUM + j];
                macc(a0[o], v0, w);
                macc(a1[o], v1, w);
            }
        }
    }
    const sf_barrett B = loadBar(bar, primeOf(m, limb));
#pragma unroll
    for (int o = 0; o < kWsumChunk; ++o) {
        if ((uint32_t)o < oc) {
            u64* dst = out + (size_t)(o0 + o) * outStride + off;
            dst[0] = sf_reduce128_acc(a0[o].lo, a0[o].hi, &B);
            dst[polyStride] = sf_reduce128_acc(a1[o].lo, a1[o].hi, &B);
        }
    }
}

struct PtrList3 {
    const u64* a[SFP_MAX_WSUM];
    const u64* c[SFP_MAX_WSUM];
    const u64* b[SFP_MAX_WSUM];
};

// out0 = sum_j a[j] * b[j], out1 = sum_j c[j] * b[j]: two coefficients per
// thread, 16-byte loads, each plaintext row read once for both polynomials.
// FP64 rows sum exact fpMulMod residues (|r| < 1.5 q < 2^43, so the up to
// SFP_MAX_WSUM terms stay below 2^50) and reduce once; the integer row (q_0)
// sums 128-bit products.  Same canonical outputs either way.
#ifndef SFHE_MAC_UNROLL
#define SFHE_MAC_UNROLL 4
#endif
constexpr int kMacUnroll = SFHE_MAC_UNROLL;  // terms per step of k_mac_plain2's FP64 loop
__global__ __launch_bounds__(kThreads) void k_mac_plain2(u64* __restrict__ out0, u64* __restrict__ out1,
                                                         const PtrList3 L, uint32_t nin, sfp_limbs m,
                                                         const sf_barrett* __restrict__ bar, uint32_t logn,
                                                         const double* __restrict__ qinvD) {
    const size_t pairs = ((size_t)m.count << logn) >> 1;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < pairs;
         i += (size_t)gridDim.x * kThreads) {
        const size_t e = 2 * i;
        const uint32_t prime = primeOf(m, (uint32_t)(e >> logn));
        const sf_barrett B = loadBar(bar, prime);
        ulonglong2 o0, o1;
        if (B.q < kFpPrimeBound) {  // (uniform per wave: a wave's 128 words lie in one row)
            const double qd = (double)B.q, qi = qinvD[prime];
            double x0 = 0.0, y0 = 0.0, x1 = 0.0, y1 = 0.0;
            uint32_t j = 0;
            auto term = [&](const ulonglong2& p, const ulonglong2& a, const ulonglong2& c) {
                const double px = u2d(p.x), py = u2d(p.y), pxq = px * qi, pyq = py * qi;
                x0 += fpMulMod(u2d(a.x), px, pxq, qd);
                y0 += fpMulMod(u2d(a.y), py, pyq, qd);
                x1 += fpMulMod(u2d(c.x), px, pxq, qd);
                y1 += fpMulMod(u2d(c.y), py, pyq, qd);
            };
            // kMacUnroll terms' 3 kMacUnroll loads in flight together (the
            // sums are exact integers: any order gives the same residues)
            for (; j + kMacUnroll <= nin; j += kMacUnroll) {
                ulonglong2 p[kMacUnroll], a[kMacUnroll], c[kMacUnroll];
#pragma unroll
                for (int u = 0; u < kMacUnroll; ++u) {
                    p[u] = *reinterpret_cast<const ulonglong2*>(L.b[j + u] + e);
                    a[u] = *reinterpret_cast<const ulonglong2*>(L.a[j + u] + e);
                    c[u] = *reinterpret_cast<const ulonglong2*>(L.c[j + u] + e);
                }
#pragma unroll
                for (int u = 0; u < kMacUnroll; ++u) term(p[u], a[u], c[u]);
            }
            for (; j + 2 <= nin; j += 2) {  // two terms' six loads in flight together
                const ulonglong2 p = *reinterpret_cast<const ulonglong2*>(L.b[j] + e);
                const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(L.a[j] + e);
                const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(L.c[j] + e);
                const ulonglong2 p2 = *reinterpret_cast<const ulonglong2*>(L.b[j + 1] + e);
                const ulonglong2 a2 = *reinterpret_cast<const ulonglong2*>(L.a[j + 1] + e);
                const ulonglong2 c2 = *reinterpret_cast<const ulonglong2*>(L.c[j + 1] + e);
                term(p, a, c);
                term(p2, a2, c2);
            }
            if (j < nin)
                term(*reinterpret_cast<const ulonglong2*>(L.b[j] + e), *reinterpret_cast<const ulonglong2*>(L.a[j] + e),
                     *reinterpret_cast<const ulonglong2*>(L.c[j] + e));
            o0.x = d2u(fpReduce(x0, qd, qi));
            o0.y = d2u(fpReduce(y0, qd, qi));
            o1.x = d2u(fpReduce(x1, qd, qi));
            o1.y = d2u(fpReduce(y1, qd, qi));
        } else {
            Acc x0{0, 0}, y0{0, 0}, x1{0, 0}, y1{0, 0};
            for (uint32_t j = 0; j < nin; ++j) {
                const ulonglong2 p = *reinterpret_cast<const ulonglong2*>(L.b[j] + e);
                const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(L.a[j] + e);
                const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(L.c[j] + e);
                macc(x0, a.x, p.x);
                macc(y0, a.y, p.y);
                macc(x1, c.x, p.x);
                macc(y1, c.y, p.y);
            }
            o0.x = sf_reduce128_acc(x0.lo, x0.hi, &B);
            o0.y = sf_reduce128_acc(y0.lo, y0.hi, &B);
            o1.x = sf_reduce128_acc(x1.lo, x1.hi, &B);
            o1.y = sf_reduce128_acc(y1.lo, y1.hi, &B);
        }
        *reinterpret_cast<ulonglong2*>(out0 + e) = o0;
        *reinterpret_cast<ulonglong2*>(out1 + e) = o1;
    }
}

// G sums of the same ciphertexts with their own plaintexts (the giant steps
// of one baby-step set, sfp_mac_plain2_multi): each a_j / c_j word is read
// once for all G, the plaintexts b[g][j] once each.  The same exact FP64
// residue sums (FP64 rows) and 128-bit sums (the integer row) as k_mac_plain2.
struct PtrListM {
    const u64* a[SFP_MAC_MULTI_N];
    const u64* c[SFP_MAC_MULTI_N];
    const u64* b[SFP_MAC_MULTI_G * SFP_MAC_MULTI_N];  // [g * nin + j]
    u64* o0[SFP_MAC_MULTI_G];
    u64* o1[SFP_MAC_MULTI_G];
};
template <int G>
__global__ __launch_bounds__(kThreads) void k_mac_plain2_multi(const PtrListM L, uint32_t nin, sfp_limbs m,
                                                               const sf_barrett* __restrict__ bar, uint32_t logn,
                                                               const double* __restrict__ qinvD) {
    const size_t pairs = ((size_t)m.count << logn) >> 1;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < pairs; i += (size_t)gridDim.x * kThreads) {
        const size_t e = 2 * i;
        const uint32_t prime = primeOf(m, (uint32_t)(e >> logn));
        const sf_barrett B = loadBar(bar, prime);
        if (B.q < kFpPrimeBound) {  // (uniform per wave)
            const double qd = (double)B.q, qi = qinvD[prime];
            double x0[G], y0[G], x1[G], y1[G];
#pragma unroll
            for (int g = 0; g < G; ++g) x0[g] = y0[g] = x1[g] = y1[g] = 0.0;
            for (uint32_t j = 0; j < nin; ++j) {
                const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(L.a[j] + e);
                const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(L.c[j] + e);
                ulonglong2 p[G];
#pragma unroll
                for (int g = 0; g < G; ++g) p[g] = *reinterpret_cast<const ulonglong2*>(L.b[g * nin + j] + e);
                const double ax = u2d(a.x), ay = u2d(a.y), cx = u2d(c.x), cy = u2d(c.y);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const double px = u2d(p[g].x), py = u2d(p[g].y), pxq = px * qi, pyq = py * qi;
                    x0[g] += fpMulMod(ax, px, pxq, qd);
                    y0[g] += fpMulMod(ay, py, pyq, qd);
                    x1[g] += fpMulMod(cx, px, pxq, qd);
                    y1[g] += fpMulMod(cy, py, pyq, qd);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                ulonglong2 o0, o1;
                o0.x = d2u(fpReduce(x0[g], qd, qi));
                o0.y = d2u(fpReduce(y0[g], qd, qi));
                o1.x = d2u(fpReduce(x1[g], qd, qi));
                o1.y = d2u(fpReduce(y1[g], qd, qi));
                *reinterpret_cast<ulonglong2*>(L.o0[g] + e) = o0;
                *reinterpret_cast<ulonglong2*>(L.o1[g] + e) = o1;
            }
        } else {  // (128-bit sums in groups of four: the integer row's registers)
#pragma unroll
            for (int h = 0; h < G; h += 4) {
                Acc x0[4], y0[4], x1[4], y1[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) x0[g] = y0[g] = x1[g] = y1[g] = Acc{0, 0};
                for (uint32_t j = 0; j < nin; ++j) {
                    const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(L.a[j] + e);
                    const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(L.c[j] + e);
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        if (h + g >= G) break;
                        const ulonglong2 p = *reinterpret_cast<const ulonglong2*>(L.b[(h + g) * nin + j] + e);
                        macc(x0[g], a.x, p.x);
                        macc(y0[g], a.y, p.y);
                        macc(x1[g], c.x, p.x);
                        macc(y1[g], c.y, p.y);
                    }
                }
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (h + g >= G) break;
                    ulonglong2 o0, o1;
                    o0.x = sf_reduce128_acc(x0[g].lo, x0[g].hi, &B);
                    o0.y = sf_reduce128_acc(y0[g].lo, y0[g].hi, &B);
                    o1.x = sf_reduce128_acc(x1[g].lo, x1[g].hi, &B);
                    o1.y = sf_reduce128_acc(y1[g].lo, y1[g].hi, &B);
                    *reinterpret_cast<ulonglong2*>(L.o0[h + g] + e) = o0;
                    *reinterpret_cast<ulonglong2*>(L.o1[h + g] + e) = o1;
                }
            }
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_mac_plain(u64* __restrict__ out, PtrList2 ab,
                                                        uint32_t nin, sfp_limbs m,
                                                        const sf_barrett* __restrict__ bar,
                                                        uint32_t logn) {
    const size_t total = (size_t)m.count << logn;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < total;
         i += (size_t)gridDim.x * kThreads) {
        const sf_barrett B = loadBar(bar, primeOf(m, (uint32_t)(i >> logn)));
        Acc acc{0, 0};
        for (uint32_t j = 0; j < nin; ++j) macc(acc, ab.a[j][i], ab.b[j][i]);
        out[i] = sf_reduce128_acc(acc.lo, acc.hi, &B);
    }
}

// out[k] = in[perm_g(k)] for every limb
struct AutArgs {
    u64* out;
    const u64* in;
    uint32_t g, count;
};
template <int NG = 1>
__global__ __launch_bounds__(kThreads) void k_automorph(const ArgSet<AutArgs, NG> S, const sf_barrett* __restrict__,
                                                        uint32_t logn) {
    const AutArgs& A = S.a[NG > 1 ? blockIdx.y : 0];
    u64* __restrict__ out = A.out;
    const u64* __restrict__ in = A.in;
    const uint32_t g = A.g, count = A.count;
    const uint32_t n = 1u << logn;
    const size_t total = (size_t)count << logn;
    const u64 mask = 2ull * n - 1;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < total;
         i += (size_t)gridDim.x * kThreads) {
        const uint32_t kk = (uint32_t)(i & (n - 1));
        const size_t row = i - kk;
        const u64 e = 2ull * sf_brev(kk, logn) + 1;
        const u64 ge = (e * g) & mask;
        const uint32_t src = sf_brev((uint32_t)((ge - 1) >> 1), logn);
        out[i] = in[row + src];
    }
}

// ============================================================================
// rescale helpers

// rows[i][x] = centred(v[x]) mod q_i   for i < cnt  (v in [0, q_last))

// out_i = (in_i - t_i) * k_i

// ============================================================================
// fast base conversion (coefficient domain)
//   out row rowOf(t) = sum_i [x_i * inv_i]_{s_i} * mod[i][t]  mod prime dst[t]
// rowOf(t) = dst[t] < Lq ? dst[t] : ell + (dst[t] - Lq)   (ext layout), or
// rowOf(t) = t when ell == 0xffffffff (dense layout).
constexpr int kMaxConvSrc = 32;

// centered != 0: each y_i is taken in (-s_i/2, s_i/2] (subtracting prod(S)
// mod t once per y_i > s_i/2), which makes the ModDown conversion error
// sum_i y_i/s_i zero-mean: a rounding, not a floor with a +K/2 bias.
// Fast base conversion of several jobs in one launch (grid: x = coefficient
// pairs, y = job, z = chunk of kConvChunk targets).  For source rows s_i
// (coefficient domain) and targets t:
//   y_i = [s_i * inv_i]_{q_i};  out_t = sum_i y_i * mod[i][t]  mod p_t
// centred: subtract prod(q_i) mod p_t once per y_i > q_i/2 (value in
// (-Q/2, Q/2] instead of [0, Q)).
#ifndef SFHE_CONV_CHUNK
#define SFHE_CONV_CHUNK 32  // targets per block; sweep on the sort: 6-16 ~ 12, 24 -0.6 ms, 32 -1.0 ms, 48 +1.1 ms
#endif
constexpr int kConvChunk = SFHE_CONV_CHUNK;
constexpr int kMaxConvJobs = 16;
constexpr int kMaxConvBig = 2;  // 60-bit sources the FP64 form splits in two
struct ConvJob {
    const u64* src;
    u64* dst;
    const uint32_t *sidx, *didx, *drow;
    const u64 *inv, *mod, *sprod;
    // FP64 form (k_convf): targets split into FP64 rows fpT[0..nFp) and
    // integer rows intT[0..nInt) (indices into the table's targets, the ones
    // below ntUse); vD/vQ [i][k] = mod[i][fpT[k]] (/ p), and for the b-th
    // 60-bit source hD/hQ [b][k] = mod[i][fpT[k]] * 2^30 mod p (/ p)
    const uint32_t *fpT, *intT;
    const double *invD, *invQ, *vD, *vQ, *hD, *hQ;
    uint32_t ns, nt, ntUse, centered, nFp, nInt, nFpAll, nbig;
};
struct ConvJobs {
    ConvJob j[kMaxConvJobs];
};

// Exact centred conversion (every centred use is a ModDown): the overflow
// v = round(sum_i y_i / s_i) of the centred y_i, estimated in FP64 with the
// oracle's operations in the oracle's order (oracle/prims_ref.c conv_rows),
// so out_t = sum_i y_i mod_i,t - v prod(S) is x's centred residue itself and
// ModDown keeps only its rounding.  yd: y_i as a correctly rounded double.
__device__ __forceinline__ double centredY(u64 y, u64 q) {
    return (double)(y > (q >> 1) ? (long long)y - (long long)q : (long long)y);
}
// out - m * sprod  (m: signed multiple count)
__device__ __forceinline__ u64 subMultiple(u64 out, long long m, u64 sprod, const sf_barrett& B) {
    if (m > 0) return sf_sub(out, bmul((u64)m, sprod, B), B.q);
    if (m < 0) return sf_add(out, bmul((u64)(-m), sprod, B), B.q);
    return out;
}

// One integer-path target row for two adjacent coefficients from canonical
// source residues ya/yb.  centred: the exact centred conversion, with the
// overflow estimates va / vb (the number of y > q/2 is added here).
template <int NS>
__device__ __forceinline__ ulonglong2 convIntTarget(const u64 (&ya)[NS], const u64 (&yb)[NS], uint32_t ns,
                                                    const u64* smodCol, int stride, const sf_barrett* sB,
                                                    const sf_barrett& B, u64 sprod, bool centred, long long va = 0,
                                                    long long vb = 0) {
    Acc s0{0, 0}, s1{0, 0};
    long long na = va, nb = vb;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        if ((uint32_t)i < ns) {
            const u64 m = smodCol[i * stride];
            macc(s0, ya[i], m);
            macc(s1, yb[i], m);
            if (centred) {
                const u64 h = sB[i].q >> 1;
                na += ya[i] > h;
                nb += yb[i] > h;
            }
        }
    }
    ulonglong2 o;
    o.x = subMultiple(sf_reduce128_acc(s0.lo, s0.hi, &B), na, sprod, B);
    o.y = subMultiple(sf_reduce128_acc(s1.lo, s1.hi, &B), nb, sprod, B);
    return o;
}

// v for two coefficients from canonical residues (integer kernels)
template <int NS>
__device__ __forceinline__ void convOverflow(const u64 (&ya)[NS], const u64 (&yb)[NS], uint32_t ns,
                                             const sf_barrett* sB, const double* sQi, long long& va, long long& vb) {
    double aa = 0.0, ab = 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i)
        if ((uint32_t)i < ns) {
            aa = fma(centredY(ya[i], sB[i].q), sQi[i], aa);
            ab = fma(centredY(yb[i], sB[i].q), sQi[i], ab);
        }
    va = (long long)rint(aa);
    vb = (long long)rint(ab);
}

// Integer form: two adjacent coefficients per thread, every constant staged
// in LDS (the output stores may alias global tables, which would otherwise
// force a reload of each per-target constant after every store).
__global__ __launch_bounds__(kThreads) void k_conv(const ConvJobs J, const sf_barrett* __restrict__ bar,
                                                   const double* __restrict__ qinvD, uint32_t logn) {
    constexpr int C = kConvChunk, NS = kMaxConvSrc;
    __shared__ u64 smod[NS * C];
    __shared__ sf_barrett sB[NS], tB[C];
    __shared__ u64 sInv[NS], tSp[C];
    __shared__ double sQi[NS];
    __shared__ uint32_t tRow[C];
    const ConvJob& c = J.j[blockIdx.y];
    const uint32_t t0 = blockIdx.z * C;
    if (t0 >= c.ntUse) return;
    const uint32_t tc = min((uint32_t)C, c.ntUse - t0);
    const uint32_t ns = c.ns;
    if (threadIdx.x < ns) {
        sB[threadIdx.x] = loadBar(bar, c.sidx[threadIdx.x]);
        sInv[threadIdx.x] = c.inv[threadIdx.x];
        sQi[threadIdx.x] = qinvD[c.sidx[threadIdx.x]];
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + tc) {
        const uint32_t k = threadIdx.x - 64, t = t0 + k;
        tB[k] = loadBar(bar, c.didx[t]);
        tSp[k] = c.sprod[t];
        tRow[k] = c.drow[t];
    }
    for (uint32_t e = threadIdx.x; e < ns * tc; e += kThreads) {
        const uint32_t i = e / tc, k = e % tc;
        smod[i * C + k] = c.mod[(size_t)i * c.nt + t0 + k];
    }
    __syncthreads();
    const uint32_t x = 2 * (blockIdx.x * kThreads + threadIdx.x);
    if (x >= (1u << logn)) return;
    u64 ya[NS], yb[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        if ((uint32_t)i < ns) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(c.src + ((size_t)i << logn) + x);
            const sf_barrett B = sB[i];
            ya[i] = bmul(v.x, sInv[i], B);
            yb[i] = bmul(v.y, sInv[i], B);
        }
    }
    long long va = 0, vb = 0;
    if (c.centered) convOverflow<NS>(ya, yb, ns, sB, sQi, va, vb);
    for (uint32_t k = 0; k < tc; ++k) {
        const ulonglong2 o = convIntTarget<NS>(ya, yb, ns, smod + k, C, sB, tB[k], tSp[k], c.centered, va, vb);
        *reinterpret_cast<ulonglong2*>(c.dst + ((size_t)tRow[k] << logn) + x) = o;
    }
}

// y = [s * inv]_q for an FP64 source, canonical or (centred) in (-q/2, q/2]
__device__ __forceinline__ double fpSourceY(u64 s, double qd, double iv, double ivq, double qi, bool centred) {
    const double y = fpReduce(fpMulMod((double)s, iv, ivq, qd), qd, qi);
    return centred && y > 0.5 * (qd - 1.0) ? y - qd : y;
}

// FP64 conversion, block-cooperative form.  A block owns kConvCoefs
// consecutive coefficients and one chunk of kConvChunk targets of one job.
// Phase 1: the block's threads compute y_i for every (source, coefficient)
// pair once (coalesced 8 B/lane loads) into LDS -- FP64 sources as exact
// doubles (signed when centred), a 60-bit source as y = yh 2^30 + yl (two
// exact doubles, the second with the multiplier mod * 2^30 mod p), and for
// integer-target blocks every source as its canonical residue.  Phase 2:
// lane = coefficient; wave w takes the target groups w, w + 4, ... of
// kConvTpi targets each: one y read from LDS feeds kConvTpi independent
// product chains, the source-major y reads are conflict-free and the
// multipliers are wave-uniform LDS broadcasts.
// Arithmetic and outputs as k_conv (canonical residues, bit-identical).
// Coefficients per block (a multiple of 64: phase 2 works on 64-coefficient
// chunks x kConvTpi-target groups).  A/B on the sort (same box): 64 / 128 /
// 256 gave 58.6 / 57.7 / 57.8 ms; smaller blocks put more of them on a CU,
// larger ones repeat phase 1 less often.
#ifndef SFHE_CONV_COEFS
#define SFHE_CONV_COEFS 128
#endif
constexpr int kConvCoefs = SFHE_CONV_COEFS;
#ifndef SFHE_CONV_TPI
#define SFHE_CONV_TPI 4
#endif
constexpr int kConvTpi = SFHE_CONV_TPI;  // FP64 targets per phase-2 iteration
// phase-1 source words per thread (NS sources x kConvCoefs coefficients)
template <int NS>
constexpr int kConvPer = (NS * kConvCoefs + kThreads - 1) / kThreads;
static_assert(kConvChunk % kConvTpi == 0 && kConvCoefs % 64 == 0 && kConvCoefs <= kThreads, "conversion block shape");

// Integer targets (the 60-bit q_0) folded into the first FP64 chunk's blocks
// of a job without 60-bit sources: up to kConvIntFold of them (a block of
// their own repeated phase 1 and added a third of the grid to a ModDown's)
constexpr uint32_t kConvIntFold = 2;
__host__ __device__ __forceinline__ bool convIntFolded(uint32_t nbig, uint32_t nFp, uint32_t nInt) {
    return nbig == 0 && nFp > 0 && nInt <= kConvIntFold;
}
template <int NS>
__global__ __launch_bounds__(kThreads) void k_convf(const ConvJobs J, const sf_barrett* __restrict__ bar,
                                                    const double* __restrict__ qinvD, uint32_t logn) {
    constexpr int C = kConvChunk, NB = kMaxConvBig, X = kConvCoefs, WAVES = kThreads / 64;
    // FP64 blocks use the multipliers (sD, sQ), integer blocks the residues
    // (smod): one LDS region serves both (4 KB less per block at NS = 16:
    // 5 blocks per CU instead of 4)
    __shared__ double sDQ[2 * NS * C];
    double* const sD = sDQ;
    double* const sQ = sDQ + NS * C;
    u64* const smod = reinterpret_cast<u64*>(sDQ);
    __shared__ double hDs[NB * C], hQs[NB * C];
    __shared__ sf_barrett sB[NS], tB[C];
    __shared__ double sInvD[NS], sInvQ[NS], sQi[NS], tQi[C];
    __shared__ u64 sInv[NS], tSp[C];
    __shared__ uint32_t tRow[C], sBig[NS];
    __shared__ u64 yL[NS * X];     // FP64 blocks: doubles' bits; integer blocks: residues
    __shared__ double yH[NB * X];  // 60-bit sources' high parts
    __shared__ double vL[X];       // centred: the overflow v of each coefficient
    __shared__ double tSpD[C], tSpQ[C];
    // the integer targets (q_0) folded into FP64 chunk 0 (convIntFolded)
    __shared__ u64 iMod[NS * kConvIntFold], iSp[kConvIntFold];
    __shared__ sf_barrett iB[kConvIntFold];
    __shared__ uint32_t iRow[kConvIntFold];
    const ConvJob& c = J.j[blockIdx.y];
    const uint32_t fpChunks = (c.nFp + C - 1) / C;
    const bool fold = convIntFolded(c.nbig, c.nFp, c.nInt);
    const bool fpBlock = blockIdx.z < fpChunks;
    if (fold && !fpBlock) return;  // (a launch's grid covers its jobs' largest z)
    const uint32_t k0 = (fpBlock ? blockIdx.z : blockIdx.z - fpChunks) * C;
    const uint32_t cnt = fpBlock ? c.nFp : c.nInt;
    if (k0 >= cnt) return;
    const uint32_t tc = min((uint32_t)C, cnt - k0);
    const uint32_t ns = c.ns;
    const uint32_t* tl = fpBlock ? c.fpT : c.intT;
    const uint32_t ti = (fold && blockIdx.z == 0) ? c.nInt : 0;  // integer targets this block adds
    // the block's source words are issued first (as k_mdrsf)
    const uint32_t x0 = blockIdx.x * X, nsX = ns * X;
    u64 sv[kConvPer<NS>];
#pragma unroll
    for (int k = 0; k < kConvPer<NS>; ++k) {
        const uint32_t e = min(threadIdx.x + k * kThreads, nsX - 1);  // (unconditional: no branch between loads)
        sv[k] = c.src[((size_t)(e / X) << logn) + x0 + e % X];
    }
    if (threadIdx.x < ns) {
        const uint32_t i = threadIdx.x, pi = c.sidx[i];
        sB[i] = loadBar(bar, pi);
        sQi[i] = qinvD[pi];
        sInv[i] = c.inv[i];
        sInvD[i] = c.invD[i];
        sInvQ[i] = c.invQ[i];
        uint32_t rank = 0;  // 60-bit sources before i (their high-part slot)
        for (uint32_t k = 0; k < i; ++k) rank += bar[c.sidx[k]].q >= kFpPrimeBound;
        sBig[i] = bar[pi].q >= kFpPrimeBound ? rank : 0xffffffffu;
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + tc) {
        const uint32_t k = threadIdx.x - 64, t = tl[k0 + k];
        tB[k] = loadBar(bar, c.didx[t]);
        tQi[k] = qinvD[c.didx[t]];
        tSp[k] = c.sprod[t];
        tSpD[k] = (double)c.sprod[t];
        tSpQ[k] = tSpD[k] / (double)tB[k].q;
        tRow[k] = c.drow[t];
    } else if (threadIdx.x >= 128 && threadIdx.x < 128 + ti) {
        const uint32_t k = threadIdx.x - 128, t = c.intT[k];
        iB[k] = loadBar(bar, c.didx[t]);
        iSp[k] = c.sprod[t];
        iRow[k] = c.drow[t];
    }
    for (uint32_t e = threadIdx.x; e < ns * ti; e += kThreads) {
        const uint32_t i = e / ti, k = e % ti;
        iMod[i * kConvIntFold + k] = c.mod[(size_t)i * c.nt + c.intT[k]];
    }
    for (uint32_t e = threadIdx.x; e < ns * tc; e += kThreads) {
        const uint32_t i = e / tc, k = e % tc;
        if (fpBlock) {
            sD[i * C + k] = c.vD[(size_t)i * c.nFpAll + k0 + k];
            sQ[i * C + k] = c.vQ[(size_t)i * c.nFpAll + k0 + k];
        } else {
            smod[i * C + k] = c.mod[(size_t)i * c.nt + tl[k0 + k]];
        }
    }
    if (fpBlock)
        for (uint32_t e = threadIdx.x; e < NB * tc; e += kThreads) {
            const uint32_t b = e / tc, k = e % tc;
            hDs[b * C + k] = c.hD[(size_t)b * c.nFpAll + k0 + k];
            hQs[b * C + k] = c.hQ[(size_t)b * c.nFpAll + k0 + k];
        }
    __syncthreads();
    const uint32_t lane = threadIdx.x % 64, w = threadIdx.x / 64;
    const bool cen = c.centered;
    // phase 1: y for every (source, coefficient) pair
#pragma unroll
    for (int k = 0; k < kConvPer<NS>; ++k) {
        const uint32_t e = threadIdx.x + k * kThreads;
        if (e >= nsX) break;
        const uint32_t i = e / X, cx = e % X;
        const u64 s = sv[k];
        const sf_barrett B = sB[i];
        if (!fpBlock) {
            yL[i * X + cx] = bmul(s, sInv[i], B);
        } else if (B.q < kFpPrimeBound) {
            yL[i * X + cx] = __double_as_longlong(fpSourceY(s, (double)B.q, sInvD[i], sInvQ[i], sQi[i], cen));
        } else {
            long long v = (long long)bmul(s, sInv[i], B);
            if (cen && v > (long long)(B.q >> 1)) v -= (long long)B.q;
            yL[i * X + cx] = __double_as_longlong((double)(v & ((1ll << 30) - 1)));
            yH[sBig[i] * X + cx] = (double)(v >> 30);
        }
    }
    __syncthreads();
    if (cen) {  // exact centred conversion: v = rint(sum_i y_i / s_i) per coefficient (convOverflow)
        for (uint32_t cx = threadIdx.x; cx < X; cx += kThreads) {
            double acc = 0.0;
#pragma unroll
            for (int i = 0; i < NS; ++i)
                if ((uint32_t)i < ns) {
                    double yd;
                    if (!fpBlock)
                        yd = centredY(yL[i * X + cx], sB[i].q);
                    else if (sBig[i] == 0xffffffffu)
                        yd = __longlong_as_double(yL[i * X + cx]);
                    else  // yh 2^30 + yl, correctly rounded as (double)(long long) y
                        yd = fma(yH[sBig[i] * X + cx], 1073741824.0, __longlong_as_double(yL[i * X + cx]));
                    acc = fma(yd, sQi[i], acc);
                }
            vL[cx] = rint(acc);
        }
        __syncthreads();
    }
    // phase 2: wave w takes coefficients [64w, 64w+64) of every target.
    // FP64 targets go kConvTpi at a time: each y read from LDS feeds
    // kConvTpi independent product chains (ILP; a quarter of the y reads).
    if (fpBlock) {
        // work items (64-coefficient chunk, group of kConvTpi targets), wave w
        // takes items w, w + WAVES, ...
        constexpr uint32_t CH = X / 64;
        const uint32_t items = CH * ((tc + kConvTpi - 1) / kConvTpi);
        for (uint32_t it = w; it < items; it += WAVES) {
            const uint32_t cx = (it % CH) * 64 + lane, k = (it / CH) * kConvTpi;
            double a[kConvTpi], pd[kConvTpi];
            const double nv = cen ? -vL[cx] : 0.0;
#pragma unroll
            for (int u = 0; u < kConvTpi; ++u) {
                const uint32_t kk = min(k + u, tc - 1);
                pd[u] = (double)tB[kk].q;
                a[u] = cen ? fpMulMod(nv, tSpD[kk], tSpQ[kk], pd[u]) : 0.0;
            }
#pragma unroll
            for (int i = 0; i < NS; ++i)
                if ((uint32_t)i < ns) {
                    const double y = __longlong_as_double(yL[i * X + cx]);
#pragma unroll
                    for (int u = 0; u < kConvTpi; ++u)
                        a[u] += fpMulMod(y, sD[i * C + k + u], sQ[i * C + k + u], pd[u]);
                }
#pragma unroll
            for (int b = 0; b < NB; ++b)
                if ((uint32_t)b < c.nbig) {
                    const double y = yH[b * X + cx];
#pragma unroll
                    for (int u = 0; u < kConvTpi; ++u)
                        a[u] += fpMulMod(y, hDs[b * C + k + u], hQs[b * C + k + u], pd[u]);
                }
#pragma unroll
            for (int u = 0; u < kConvTpi; ++u)
                if (k + u < tc)
                    c.dst[((size_t)tRow[k + u] << logn) + x0 + cx] = (u64)fpReduce(a[u], pd[u], tQi[k + u]);
        }
        // the folded integer targets: canonical residues of the FP64 y's
        // (no 60-bit sources here), as an integer block computes them
        for (uint32_t kc = w * 64; kc < ti * X; kc += WAVES * 64) {
            const uint32_t k = kc / X, cx = kc % X + lane;
            const sf_barrett B = iB[k];
            Acc s0{0, 0};
            long long neg = cen ? (long long)vL[cx] : 0;
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                if ((uint32_t)i < ns) {
                    const double y = __longlong_as_double(yL[i * X + cx]);
                    macc(s0, (u64)(y < 0.0 ? y + (double)sB[i].q : y), iMod[i * kConvIntFold + k]);
                    neg += cen && y < 0.0;
                }
            }
            c.dst[((size_t)iRow[k] << logn) + x0 + cx] = subMultiple(sf_reduce128_acc(s0.lo, s0.hi, &B), neg, iSp[k], B);
        }
        return;
    }
    for (uint32_t kc = w * 64; kc < tc * X; kc += WAVES * 64) {  // integer targets, one at a time
        const uint32_t k = kc / X, cx = kc % X + lane;
        const sf_barrett B = tB[k];
        u64 out;
        {
            Acc s0{0, 0};
            long long neg = cen ? (long long)vL[cx] : 0;
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                if ((uint32_t)i < ns) {
                    const u64 y = yL[i * X + cx];
                    macc(s0, y, smod[i * C + k]);
                    neg += cen && y > (sB[i].q >> 1);
                }
            }
            out = subMultiple(sf_reduce128_acc(s0.lo, s0.hi, &B), neg, tSp[k], B);
        }
        c.dst[((size_t)tRow[k] << logn) + x0 + cx] = out;
    }
}

// ModDown conversion fused with the following rescale (sfp_moddown_rescale).
// Per coefficient x of each poly: the centred P->Q conversion conv_t of the K
// P-rows (as k_conv), the dropped row's coefficient r = (a_l - conv_l) P^-1
// mod q_l, and for every kept target t < l:  y_t = conv_t + P_t [r]_t, with
// [r]_t the centred lift of r (r > q_l/2 stands for r - q_l).
constexpr int kMdrsJobs = 16;
struct MdrsJob {
    const u64* src;  // K P-rows, coefficient domain
    const u64* al;   // accumulator row l, coefficient domain
    u64* dst;        // l rows
};
struct MdrsArgs {
    MdrsJob j[kMdrsJobs];  // blockIdx.y: two polys, or the polys of up to four merged launches
    const uint32_t* sidx;
    const u64 *inv, *mod, *sprod;  // the ModDown conversion table (targets 0..)
    const u64 *pmod, *lsub;        // P mod q_t, q_l mod q_t
    // FP64 form (k_mdrsf): the table's FP64 companions (target rows fpT /
    // intT as in ConvJob, restricted to t < l), the dropped row's column
    // (lD/lQ [i * nFpAll] = mod[i][l] (/ q_l)) and P mod q_t as doubles
    const uint32_t *fpT, *intT;
    const double *invD, *invQ, *vD, *vQ, *lD, *lQ, *pmodD, *pmodQ;
    u64 pinvl;                     // P^-1 mod q_l
    uint32_t ns, nt, l, nFp, nInt, nFpAll;
};

// Integer form, two coefficients per thread, constants in LDS.
__global__ __launch_bounds__(kThreads) void k_conv_mdrs(const MdrsArgs A, const sf_barrett* __restrict__ bar,
                                                        const double* __restrict__ qinvD, uint32_t logn) {
    constexpr int C = kConvChunk, W = C + 1, NS = kMaxConvSrc;  // column C: the dropped row l
    __shared__ u64 smod[NS * W];
    __shared__ sf_barrett sB[NS], tB[W];
    __shared__ u64 sInv[NS], tSp[W], tPm[W], tLs[W];
    __shared__ double sQi[NS];
    const MdrsJob& J = A.j[blockIdx.y];
    const uint32_t t0 = blockIdx.z * C;
    if (t0 >= A.l) return;
    const uint32_t tc = min((uint32_t)C, A.l - t0);
    const uint32_t ns = A.ns;
    if (threadIdx.x < ns) {
        sB[threadIdx.x] = loadBar(bar, A.sidx[threadIdx.x]);
        sInv[threadIdx.x] = A.inv[threadIdx.x];
        sQi[threadIdx.x] = qinvD[A.sidx[threadIdx.x]];
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + W && (threadIdx.x - 64 < tc || threadIdx.x - 64 == C)) {
        const uint32_t k = threadIdx.x - 64, tt = k < tc ? t0 + k : A.l;
        tB[k] = loadBar(bar, tt);
        tSp[k] = A.sprod[tt];
        if (k < tc) {
            tPm[k] = A.pmod[tt];
            tLs[k] = A.lsub[tt];
        }
    }
    for (uint32_t e = threadIdx.x; e < ns * W; e += kThreads) {
        const uint32_t i = e / W, k = e % W;
        const bool use = k < tc || k == (uint32_t)C;
        smod[e] = use ? A.mod[(size_t)i * A.nt + (k < tc ? t0 + k : A.l)] : 0;
    }
    __syncthreads();
    const uint32_t x = 2 * (blockIdx.x * kThreads + threadIdx.x);
    if (x >= (1u << logn)) return;
    u64 ya[NS], yb[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        if ((uint32_t)i < ns) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(J.src + ((size_t)i << logn) + x);
            const sf_barrett B = sB[i];
            ya[i] = bmul(v.x, sInv[i], B);
            yb[i] = bmul(v.y, sInv[i], B);
        }
    }
    long long va, vb;
    convOverflow<NS>(ya, yb, ns, sB, sQi, va, vb);
    // the dropped row: r = (a_l - conv_l) * P^-1 mod q_l
    const sf_barrett BL = tB[C];
    const ulonglong2 cl = convIntTarget<NS>(ya, yb, ns, smod + C, W, sB, BL, tSp[C], true, va, vb);
    const ulonglong2 al = *reinterpret_cast<const ulonglong2*>(J.al + ((size_t)A.l << logn) + x);
    const u64 ra = bmul(sf_sub(al.x, cl.x, BL.q), A.pinvl, BL), rb = bmul(sf_sub(al.y, cl.y, BL.q), A.pinvl, BL);
    const bool na = ra > (BL.q >> 1), nb = rb > (BL.q >> 1);
    for (uint32_t k = 0; k < tc; ++k) {
        const sf_barrett B = tB[k];
        ulonglong2 v = convIntTarget<NS>(ya, yb, ns, smod + k, W, sB, B, tSp[k], true, va, vb);
        u64 la = sf_reduce128(ra, 0, &B), lb = sf_reduce128(rb, 0, &B);
        if (na) la = sf_sub(la, tLs[k], B.q);
        if (nb) lb = sf_sub(lb, tLs[k], B.q);
        v.x = sf_add(v.x, bmul(la, tPm[k], B), B.q);
        v.y = sf_add(v.y, bmul(lb, tPm[k], B), B.q);
        *reinterpret_cast<ulonglong2*>(J.dst + ((size_t)(t0 + k) << logn) + x) = v;
    }
}

// Integer form, block-cooperative as k_mdrsf (round 6: k_conv_mdrs, one
// thread per coefficient pair with every source in registers, took 424 VGPRs
// and 18.7 % of the k-way sort at one wave per SIMD, profiles/r06/): for
// tables whose sources the FP64 forms cannot take (the scale-59 chains' 60-bit
// P primes).  A block owns kConvCoefs coefficients of one polynomial and one
// chunk of kConvChunk targets.  Phase 1: the canonical y_i of every (source,
// coefficient) pair into LDS.  Then one thread per coefficient: the overflow
// v (convOverflow's operations in its order), the count of centred y_i, and
// the dropped row's r = (a_l - conv_l) P^-1 mod q_l.  Phase 2: one lane per
// coefficient and target, the 128-bit sum over the sources from LDS.  The
// same integers as k_conv_mdrs, so the same outputs.
template <int NS>
__global__ __launch_bounds__(kThreads) void k_mdrsi(const MdrsArgs A, const sf_barrett* __restrict__ bar,
                                                    const double* __restrict__ qinvD, uint32_t logn) {
    constexpr int C = kConvChunk, X = kConvCoefs, WAVES = kThreads / 64;
    __shared__ u64 smod[NS * C];  // mod[i][t] of this chunk's targets
    __shared__ u64 sLm[NS];       // mod[i][l]
    __shared__ sf_barrett sB[NS], tB[C];
    __shared__ u64 sInv[NS], tSp[C], tPm[C], tLs[C];
    __shared__ double sQi[NS];
    __shared__ u64 yL[NS * X];     // canonical y_i
    __shared__ u64 rL[X];          // the dropped row's r, canonical mod q_l
    __shared__ long long nL[X];    // v + #{y_i > s_i / 2}: the multiple of prod(S) the centred sum drops
    const MdrsJob& J = A.j[blockIdx.y];
    const uint32_t k0 = blockIdx.z * C;
    if (k0 >= A.l) return;
    const uint32_t tc = min((uint32_t)C, A.l - k0);
    const uint32_t ns = A.ns, x0 = blockIdx.x * X, nsX = ns * X;
    // the block's source words and its dropped-row words first (one round trip)
    u64 sv[kConvPer<NS>];
#pragma unroll
    for (int k = 0; k < kConvPer<NS>; ++k) {
        const uint32_t e = min(threadIdx.x + k * kThreads, nsX - 1);  // (unconditional: no branch between loads)
        sv[k] = J.src[((size_t)(e / X) << logn) + x0 + e % X];
    }
    const u64 alv = J.al[((size_t)A.l << logn) + x0 + threadIdx.x % X];
    const sf_barrett BL = loadBar(bar, A.l);
    const u64 sprl = A.sprod[A.l];
    if (threadIdx.x < ns) {
        const uint32_t i = threadIdx.x, pi = A.sidx[i];
        sB[i] = loadBar(bar, pi);
        sInv[i] = A.inv[i];
        sQi[i] = qinvD[pi];
        sLm[i] = A.mod[(size_t)i * A.nt + A.l];
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + tc) {
        const uint32_t k = threadIdx.x - 64, t = k0 + k;
        tB[k] = loadBar(bar, t);
        tSp[k] = A.sprod[t];
        tPm[k] = A.pmod[t];
        tLs[k] = A.lsub[t];
    }
    for (uint32_t e = threadIdx.x; e < ns * tc; e += kThreads) {
        const uint32_t i = e / tc, k = e % tc;
        smod[i * C + k] = A.mod[(size_t)i * A.nt + k0 + k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kConvPer<NS>; ++k) {
        const uint32_t e = threadIdx.x + k * kThreads;
        if (e < nsX) {
            const uint32_t i = e / X;
            yL[e] = bmul(sv[k], sInv[i], sB[i]);
        }
    }
    __syncthreads();
    if (threadIdx.x < X) {
        const uint32_t cx = threadIdx.x;
        double aa = 0.0;
        long long cnt = 0;
        Acc sl{0, 0};
#pragma unroll
        for (int i = 0; i < NS; ++i)
            if ((uint32_t)i < ns) {
                const u64 y = yL[i * X + cx];
                aa = fma(centredY(y, sB[i].q), sQi[i], aa);
                cnt += y > (sB[i].q >> 1);
                macc(sl, y, sLm[i]);
            }
        const long long na = (long long)rint(aa) + cnt;
        nL[cx] = na;
        const u64 cl = subMultiple(sf_reduce128_acc(sl.lo, sl.hi, &BL), na, sprl, BL);
        rL[cx] = bmul(sf_sub(alv, cl, BL.q), A.pinvl, BL);
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x % 64, w = threadIdx.x / 64;
    const u64 lhalf = BL.q >> 1;
    for (uint32_t kc = w * 64; kc < tc * X; kc += WAVES * 64) {
        const uint32_t k = kc / X, cx = kc % X + lane;
        const sf_barrett B = tB[k];
        Acc s0{0, 0};
#pragma unroll
        for (int i = 0; i < NS; ++i)
            if ((uint32_t)i < ns) macc(s0, yL[i * X + cx], smod[i * C + k]);
        u64 out = subMultiple(sf_reduce128_acc(s0.lo, s0.hi, &B), nL[cx], tSp[k], B);
        const u64 r = rL[cx];
        u64 lift = sf_reduce128(r, 0, &B);
        if (r > lhalf) lift = sf_sub(lift, tLs[k], B.q);
        out = sf_add(out, bmul(lift, tPm[k], B), B.q);
        J.dst[((size_t)(k0 + k) << logn) + x0 + cx] = out;
    }
}

// FP64 form of k_conv_mdrs, block-cooperative as k_convf: every source (P
// row) and the dropped row's prime below kFpPrimeBound.  Phase 1: the
// centred y_i of every (source, coefficient) pair into LDS; then wave 0 forms
// each coefficient's dropped-row value r = (a_l - conv_l) P^-1 mod q_l
// (centred).  Phase 2: FP64 targets fold [r]_t P_t into the conversion sum;
// integer targets (fpT / intT split as in k_convf) use canonical residues.
// BIGL: the dropped row's prime is 60-bit (scale-59 chains: the k-way /
// bootstrapping contexts) and every target below it an integer row: r is
// formed in integer arithmetic (k_conv_mdrs's), kept as its canonical
// residue, and only integer blocks run.
// Integer targets (the 60-bit q_0) of a ModDown+rescale folded into its
// first FP64 chunk's blocks: up to kMdrsIntFold of them, with at least one
// FP64 chunk (host and kernel decide it alike)
constexpr uint32_t kMdrsIntFold = 2;
__host__ __device__ __forceinline__ bool mdrsIntFolded(bool bigl, uint32_t nFp, uint32_t nInt) {
    return !bigl && nFp > 0 && nInt <= kMdrsIntFold;
}
template <int NS, bool BIGL = false>
__global__ __launch_bounds__(kThreads) void k_mdrsf(const MdrsArgs A, const sf_barrett* __restrict__ bar,
                                                    const double* __restrict__ qinvD, uint32_t logn) {
    constexpr int C = kConvChunk, X = kConvCoefs, WAVES = kThreads / 64;
    // one LDS region for the FP64 multipliers or the integer residues (as k_convf)
    __shared__ double sDQ[2 * NS * C];
    double* const sD = sDQ;
    double* const sQ = sDQ + NS * C;
    u64* const smod = reinterpret_cast<u64*>(sDQ);
    __shared__ double sLD[NS], sLQ[NS];
    __shared__ u64 sLm[NS];  // BIGL: mod[i][l]
    __shared__ sf_barrett sB[NS], tB[C];
    __shared__ double sInvD[NS], sInvQ[NS], sQi[NS], tQi[C], tPd[C], tPq[C];
    __shared__ u64 tSp[C], tPm[C], tLs[C];
    __shared__ uint32_t tRow[C];
    __shared__ double yL[NS * X], rL[X], vL[X];
    __shared__ double tSpD[C], tSpQ[C];
    // the integer targets (q_0) folded into FP64 chunk 0 (mdrsIntFolded): a
    // block of their own repeated phase 1 and doubled a small ModDown's grid
    __shared__ u64 iMod[NS * kMdrsIntFold], iSp[kMdrsIntFold], iPm[kMdrsIntFold], iLs[kMdrsIntFold];
    __shared__ sf_barrett iB[kMdrsIntFold];
    __shared__ uint32_t iRow[kMdrsIntFold];
    const MdrsJob& J = A.j[blockIdx.y];
    const uint32_t fpChunks = (A.nFp + C - 1) / C;
    const bool fold = mdrsIntFolded(BIGL, A.nFp, A.nInt);
    const bool fpBlock = blockIdx.z < fpChunks;
    if (fold && !fpBlock) return;
    const uint32_t k0 = (fpBlock ? blockIdx.z : blockIdx.z - fpChunks) * C;
    const uint32_t cnt = fpBlock ? A.nFp : A.nInt;
    if (k0 >= cnt) return;
    const uint32_t tc = min((uint32_t)C, cnt - k0);
    const uint32_t ns = A.ns;
    const uint32_t* tl = fpBlock ? A.fpT : A.intT;
    const uint32_t ti = (fold && blockIdx.z == 0) ? A.nInt : 0;  // integer targets this block adds
    // the block's source words and its dropped-row words are issued first, so
    // their HBM latency overlaps the constant staging below (one round trip
    // for the whole phase 1 instead of one per loop iteration)
    const uint32_t x0 = blockIdx.x * X, nsX = ns * X;
#ifdef SFHE_NTT_TRACE
    unsigned long long tprev = clock64(), tacc[4] = {0, 0, 0, 0};
#define MDRS_MARK(i)                                 \
    {                                                \
        const unsigned long long t_ = clock64();     \
        tacc[(i)] += t_ - tprev;                     \
        tprev = t_;                                  \
    }
#define MDRS_FLUSH()                                                                       \
    if (threadIdx.x == 0) {                                                                \
        auto& slot = g_mdrsTrace[(blockIdx.x + blockIdx.y * gridDim.x) % kTraceSlots];     \
        for (int i_ = 0; i_ < 4; ++i_) atomicAdd(&slot[i_], tacc[i_]);                     \
        atomicAdd(&slot[7], 1ull);                                                         \
    }
#else
#define MDRS_MARK(i)
#define MDRS_FLUSH()
#endif
    u64 sv[kConvPer<NS>];
#pragma unroll
    for (int k = 0; k < kConvPer<NS>; ++k) {
        const uint32_t e = min(threadIdx.x + k * kThreads, nsX - 1);  // (unconditional: no branch between loads)
        sv[k] = J.src[((size_t)(e / X) << logn) + x0 + e % X];
    }
    const u64 alv = J.al[((size_t)A.l << logn) + x0 + threadIdx.x % X];
    // the dropped row's constants, issued with the loads above (read after
    // the second barrier, they were a round trip of their own)
    const u64 qlq = bar[A.l].q, sprl = A.sprod[A.l];
    const double qliD = qinvD[A.l];
    if (threadIdx.x < ns) {
        const uint32_t i = threadIdx.x, pi = A.sidx[i];
        sB[i] = loadBar(bar, pi);
        sQi[i] = qinvD[pi];
        sInvD[i] = A.invD[i];
        sInvQ[i] = A.invQ[i];
        if (BIGL) {
            sLm[i] = A.mod[(size_t)i * A.nt + A.l];
        } else {
            sLD[i] = A.lD[(size_t)i * A.nFpAll];
            sLQ[i] = A.lQ[(size_t)i * A.nFpAll];
        }
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + tc) {
        const uint32_t k = threadIdx.x - 64, t = tl[k0 + k];
        tB[k] = loadBar(bar, t);
        tQi[k] = qinvD[t];
        tSp[k] = A.sprod[t];
        tSpD[k] = (double)A.sprod[t];
        tSpQ[k] = tSpD[k] / (double)tB[k].q;
        tPm[k] = A.pmod[t];
        tLs[k] = A.lsub[t];
        if (!BIGL) {
            tPd[k] = A.pmodD[t];
            tPq[k] = A.pmodQ[t];
        }
        tRow[k] = t;
    } else if (threadIdx.x >= 128 && threadIdx.x < 128 + ti) {
        const uint32_t k = threadIdx.x - 128, t = A.intT[k];
        iB[k] = loadBar(bar, t);
        iSp[k] = A.sprod[t];
        iPm[k] = A.pmod[t];
        iLs[k] = A.lsub[t];
        iRow[k] = t;
    }
    for (uint32_t e = threadIdx.x; e < ns * ti; e += kThreads) {
        const uint32_t i = e / ti, k = e % ti;
        iMod[i * kMdrsIntFold + k] = A.mod[(size_t)i * A.nt + A.intT[k]];
    }
    for (uint32_t e = threadIdx.x; e < ns * tc; e += kThreads) {
        const uint32_t i = e / tc, k = e % tc;
        if (fpBlock) {
            sD[i * C + k] = A.vD[(size_t)i * A.nFpAll + k0 + k];
            sQ[i * C + k] = A.vQ[(size_t)i * A.nFpAll + k0 + k];
        } else {
            smod[i * C + k] = A.mod[(size_t)i * A.nt + tl[k0 + k]];
        }
    }
    __syncthreads();
    MDRS_MARK(0);
    const uint32_t lane = threadIdx.x % 64, w = threadIdx.x / 64;
#pragma unroll
    for (int k = 0; k < kConvPer<NS>; ++k) {
        const uint32_t e = threadIdx.x + k * kThreads;
        if (e < nsX) {
            const uint32_t i = e / X;
            yL[e] = fpSourceY(sv[k], (double)sB[i].q, sInvD[i], sInvQ[i], sQi[i], true);
        }
    }
    __syncthreads();
    MDRS_MARK(1);
    const double qld = (double)qlq;
    if (threadIdx.x < X) {  // the dropped row: r = (a_l - conv_l) * P^-1 mod q_l, centred
        const uint32_t cx = threadIdx.x;
        // exact centred conversion: the overflow v (convOverflow), removed from every target
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i)
            if ((uint32_t)i < ns) acc = fma(yL[i * X + cx], sQi[i], acc);
        const double v = rint(acc);
        vL[cx] = v;
        if (BIGL) {  // as k_conv_mdrs: canonical y, the count of negative ones
            const sf_barrett BL = loadBar(bar, A.l);
            Acc sl{0, 0};
            long long neg = (long long)v;
#pragma unroll
            for (int i = 0; i < NS; ++i)
                if ((uint32_t)i < ns) {
                    const double y = yL[i * X + cx];
                    macc(sl, (u64)(y < 0.0 ? y + (double)sB[i].q : y), sLm[i]);
                    neg += y < 0.0;
                }
            const u64 cl = subMultiple(sf_reduce128_acc(sl.lo, sl.hi, &BL), neg, A.sprod[A.l], BL);
            rL[cx] = __longlong_as_double((long long)bmul(sf_sub(alv, cl, BL.q), A.pinvl, BL));
        } else {
        const double spl = (double)sprl;
        double cl = fpMulMod(-v, spl, spl / qld, qld);
#pragma unroll
        for (int i = 0; i < NS; ++i)
            if ((uint32_t)i < ns) cl += fpMulMod(yL[i * X + cx], sLD[i], sLQ[i], qld);
        const double qli = qliD;
        const double pl = (double)A.pinvl;
        rL[cx] = fpSourceY((u64)fpReduce((double)alv - fpReduce(cl, qld, qli), qld, qli), qld, pl, pl / qld, qli,
                           true);
        }
    }
    __syncthreads();
    MDRS_MARK(2);
    // integer targets, one at a time: this block's own (an integer chunk), or
    // the folded ones after the FP64 targets
    auto intTargets = [&](uint32_t cntT, const sf_barrett* TB, const u64* SM, uint32_t smStride, const u64* TSP,
                          const u64* TPM, const u64* TLS, const uint32_t* TROW) {
        for (uint32_t kc = w * 64; kc < cntT * X; kc += WAVES * 64) {
            const uint32_t k = kc / X, cx = kc % X + lane;
            const double r = rL[cx];
            u64 out;
            {
                const sf_barrett B = TB[k];
                Acc s0{0, 0};
                long long neg = (long long)vL[cx];
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    if ((uint32_t)i < ns) {
                        const double y = yL[i * X + cx];
                        macc(s0, (u64)(y < 0.0 ? y + (double)sB[i].q : y), SM[i * smStride + k]);
                        neg += y < 0.0;
                    }
                }
                out = subMultiple(sf_reduce128_acc(s0.lo, s0.hi, &B), neg, TSP[k], B);
                u64 lift;
                bool rneg;
                if (BIGL) {  // canonical residue; centred: > q_l / 2 stands for r - q_l
                    const u64 rc = (u64)__double_as_longlong(r);
                    rneg = rc > (bar[A.l].q >> 1);
                    lift = sf_reduce128(rc, 0, &B);
                } else {
                    rneg = r < 0.0;
                    lift = sf_reduce128((u64)(r < 0.0 ? r + qld : r), 0, &B);
                }
                if (rneg) lift = sf_sub(lift, TLS[k], B.q);
                out = sf_add(out, bmul(lift, TPM[k], B), B.q);
            }
            J.dst[((size_t)TROW[k] << logn) + x0 + cx] = out;
        }
    };
    if (!BIGL && fpBlock) {  // kConvTpi targets at a time, work items as k_convf
        constexpr uint32_t CH = X / 64;
        const uint32_t items = CH * ((tc + kConvTpi - 1) / kConvTpi);
        for (uint32_t it = w; it < items; it += WAVES) {
            const uint32_t cx = (it % CH) * 64 + lane, k = (it / CH) * kConvTpi;
            const double r = rL[cx], nv = -vL[cx];
            double a[kConvTpi], pd[kConvTpi];
#pragma unroll
            for (int u = 0; u < kConvTpi; ++u) {
                const uint32_t kk = min(k + u, tc - 1);
                pd[u] = (double)tB[kk].q;
                a[u] = fpMulMod(r, tPd[kk], tPq[kk], pd[u]) + fpMulMod(nv, tSpD[kk], tSpQ[kk], pd[u]);
            }
#pragma unroll
            for (int i = 0; i < NS; ++i)
                if ((uint32_t)i < ns) {
                    const double y = yL[i * X + cx];
#pragma unroll
                    for (int u = 0; u < kConvTpi; ++u)
                        a[u] += fpMulMod(y, sD[i * C + k + u], sQ[i * C + k + u], pd[u]);
                }
#pragma unroll
            for (int u = 0; u < kConvTpi; ++u)
                if (k + u < tc)
                    J.dst[((size_t)tRow[k + u] << logn) + x0 + cx] = (u64)fpReduce(a[u], pd[u], tQi[k + u]);
        }
        if (ti) intTargets(ti, iB, iMod, kMdrsIntFold, iSp, iPm, iLs, iRow);
        MDRS_MARK(3);
        MDRS_FLUSH();
        return;
    }
    intTargets(tc, tB, smod, C, tSp, tPm, tLs, tRow);
}
#undef MDRS_MARK
#undef MDRS_FLUSH

// ModDown's conversion -- and the rescale fused with it -- in the forward
// COL pass of its output rows (sfp_moddown2 / sfp_moddown_rescale, ring
// 2^16).  The INTT of the P rows (and the rescale's dropped row) folds the
// conversion's factors (P/p_i)^-1 into its last pass and stores its FP64 rows
// as doubles (mdPost), so y_i = x_i (P/p_i)^-1 mod p_i arrives ready to be
// centred.  A block owns one COL tile of kModdownTg target rows t of one
// polynomial: it reads that tile of each of the K y rows (L2 hits for every
// target group after the first), centres them, and accumulates as it goes each
// FP64 target's conversion sum, the overflow v = rint(sum_i y_i / p_i) and,
// with the rescale, the dropped row's conversion; then r = (a_l - conv_l)
// P^-1 mod q_l (centred), and each target's tile
//   y_t = conv_t - v [P]_t (+ [r]_t pmod_t)
// runs its COL rounds in LDS and is stored.  The converted rows are never
// written and read back, and k_mdrsf / k_convf's ModDown launch is gone.
// The same integers as those kernels (exact FP64 sums of fpMulMod residues;
// the integer row q_0 in 128-bit sums of canonical y), so the same outputs.
struct MdColArgs {
    const uint32_t* sidx;       // source primes [ns]
    const double *invD, *invQ;  // [ns]: the table's inv_i as a double, / p_i
    const double *mD, *mQ;      // [ns][nt]: mod[i][t] as a double, / q_t
    const u64* mI;              // [ns][nt]: mod[i][t] (the integer target)
    const u64* sprod;           // [nt]: prod(P) mod q_t
    const double *spD, *spQ;    // [nt]: as a double, / q_t
    const u64 *pmod, *lsub;     // rescale [l]: pmod_t, q_l mod q_t
    const double *pmD, *pmQ;    // rescale [l]: pmod_t as a double, / q_t
    u64 pinvl;                  // rescale: P^-1 mod q_l
    uint32_t ns, nt, l, rs;     // rs: with the rescale (targets t < l)
};
#ifndef SFHE_MODDOWN_TG
#define SFHE_MODDOWN_TG 4
#endif
constexpr int kModdownTg = SFHE_MODDOWN_TG;

// a source word as the INTT left it (the conversion's factor folded into its
// last pass: a canonical residue stored as a double) -> the centred y_i
__device__ __forceinline__ double mdCentred(u64 bits, double q, double half) {
    const double y = __longlong_as_double(bits);
    return y > half ? y - q : y;
}

template <int TILE, int NG, int TG>
__global__ __launch_bounds__(TILE >> 2) void k_moddown_col(const RowGroupSet<NG> GS, const sf_barrett* __restrict__ bar,
                                                           const u64* __restrict__ tw, const u64* __restrict__ twS,
                                                           const u64* __restrict__, const u64* __restrict__,
                                                           uint32_t logn, const double* __restrict__ twD,
                                                           const double* __restrict__ qinvD,
                                                           const double* __restrict__, const double* __restrict__, int,
                                                           const double* __restrict__) {
    constexpr int LE = 2, NT = TILE >> LE, NPAIR = (1 << LE) / 2, W4 = 2 * NPAIR;
    __shared__ u64 s[TILE];
    __shared__ u64 tW[kNttColTw], tX[kNttColTw];
    const uint32_t n = 1u << logn;
    const uint32_t logR = logn - 8;  // (8: ring 2^16, checked on the host)
    uint32_t rid;
    const RowGroup& G = GS.a[argSel(GS, rid)];
    const MdColArgs& A = *G.md;
    const uint32_t RG = (G.R + TG - 1) / TG;
    const uint32_t pp = rid / RG, g0 = (rid % RG) * TG;
    NttTile T;
    T.logn = logn;
    T.d = logR;
    T.logC = (uint32_t)__builtin_ctz(TILE) - logR;
    T.C = 1u << T.logC;
    const uint32_t tile = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    T.c0 = tile * T.C;
    T.r0 = 0;
    auto tileOff = [&](int k) -> size_t {
        const uint32_t e = 2 * (threadIdx.x + k * NT);
        return (size_t)(e >> T.logC) * 256 + T.c0 + (e & (T.C - 1));
    };
    const uint32_t ns = A.ns, nt = A.nt, l = A.l;
    const bool rs = A.rs != 0;
    bool live[TG];
    uint32_t prime[TG];
    double qd[TG], qi[TG];
    bool fpT[TG];
#pragma unroll
    for (int u = 0; u < TG; ++u) {
        live[u] = g0 + u < G.R;
        prime[u] = primeOf(G.pm, min(g0 + u, G.R - 1));
        const u64 q = bar[prime[u]].q;
        fpT[u] = q < kFpPrimeBound;
        qd[u] = (double)q;
        qi[u] = qinvD[prime[u]];
    }
    const double qld = rs ? (double)bar[l].q : 1.0;
    double acc[TG][W4], vacc[W4], cacc[W4];
#pragma unroll
    for (int w = 0; w < W4; ++w) {
        vacc[w] = 0.0;
        cacc[w] = 0.0;
#pragma unroll
        for (int u = 0; u < TG; ++u) acc[u][w] = 0.0;
    }
    constexpr int GRP = 4;  // source tiles in flight together
    for (uint32_t s0 = 0; s0 < ns; s0 += GRP) {
        ulonglong2 v[GRP][NPAIR];
#pragma unroll
        for (int g = 0; g < GRP; ++g)
            if (s0 + g < ns)
#pragma unroll
                for (int k = 0; k < NPAIR; ++k)
                    v[g][k] = *reinterpret_cast<const ulonglong2*>(rowAt(G.copy, pp, s0 + g) + tileOff(k));
#pragma unroll
        for (int g = 0; g < GRP; ++g) {
            const uint32_t sI = s0 + g;
            if (sI >= ns) break;
            const uint32_t pi = A.sidx[sI];
            const double sq = (double)bar[pi].q, sqi = qinvD[pi], half = 0.5 * (sq - 1.0);
            double y[W4];
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {
                y[2 * k] = mdCentred(v[g][k].x, sq, half);
                y[2 * k + 1] = mdCentred(v[g][k].y, sq, half);
            }
            const size_t mrow = (size_t)sI * nt;
#pragma unroll
            for (int w = 0; w < W4; ++w) vacc[w] = fma(y[w], sqi, vacc[w]);  // (k_mdrsf's order: i ascending)
            if (rs) {
                const double md = A.mD[mrow + l], mq = A.mQ[mrow + l];
#pragma unroll
                for (int w = 0; w < W4; ++w) cacc[w] += fpMulMod(y[w], md, mq, qld);
            }
#pragma unroll
            for (int u = 0; u < TG; ++u) {
                if (!live[u] || !fpT[u]) continue;
                const double md = A.mD[mrow + g0 + u], mq = A.mQ[mrow + g0 + u];
#pragma unroll
                for (int w = 0; w < W4; ++w) acc[u][w] += fpMulMod(y[w], md, mq, qd[u]);
            }
        }
    }
    double vv[W4], rr[W4];
#pragma unroll
    for (int w = 0; w < W4; ++w) {
        vv[w] = rint(vacc[w]);
        rr[w] = 0.0;
    }
    if (rs) {  // the dropped row: r = (a_l - conv_l) P^-1 mod q_l, centred
        const u64* al = rowAt(G.pre, pp, 0);
        const double spl = (double)A.sprod[l], qli = qinvD[l], pl = (double)A.pinvl;
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) {
            const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(al + tileOff(k));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int w = 2 * k + h;
                const double cl = fpMulMod(-vv[w], spl, spl / qld, qld) + cacc[w];
                const double av = __longlong_as_double(h ? a.y : a.x);
                rr[w] = fpSourceY((u64)fpReduce(av - fpReduce(cl, qld, qli), qld, qli), qld, pl, pl / qld, qli, true);
            }
        }
    }
    constexpr int kColPer = (int)((kNttColTw + NT - 1) / NT);
    const uint32_t colTw = (1u << logR) - 1;
    bool first = true;
    // FP64 targets first (their sums die there), then the integer row, whose
    // 128-bit sums then do not share registers with them
#pragma unroll
    for (int ph = 0; ph < 2; ++ph)
#pragma unroll
    for (int u = 0; u < TG; ++u) {
        if (!live[u] || fpT[u] != (ph == 0)) continue;
        const uint32_t t = g0 + u, pr = prime[u];
        const bool fp = ph == 0;
        const u64 q = bar[pr].q;
        ulonglong2 xr[NPAIR];
        if (fp) {
            const double spd = A.spD[t], spq = A.spQ[t];
            const double pmd = rs ? A.pmD[t] : 0.0, pmq = rs ? A.pmQ[t] : 0.0;
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {
                double a0 = acc[u][2 * k] + fpMulMod(-vv[2 * k], spd, spq, qd[u]);
                double a1 = acc[u][2 * k + 1] + fpMulMod(-vv[2 * k + 1], spd, spq, qd[u]);
                if (rs) {
                    a0 += fpMulMod(rr[2 * k], pmd, pmq, qd[u]);
                    a1 += fpMulMod(rr[2 * k + 1], pmd, pmq, qd[u]);
                }
                xr[k].x = __double_as_longlong(fpReduce(a0, qd[u], qi[u]));
                xr[k].y = __double_as_longlong(fpReduce(a1, qd[u], qi[u]));
            }
        } else {  // the integer row (q_0): 128-bit sums of the canonical y, sources re-read (L2)
            const sf_barrett CB = loadBar(bar, pr);
            Acc a2[W4];
            long long neg[W4];
#pragma unroll
            for (int w = 0; w < W4; ++w) {
                a2[w] = Acc{0, 0};
                neg[w] = (long long)vv[w];
            }
            for (uint32_t sI = 0; sI < ns; ++sI) {
                const uint32_t pi = A.sidx[sI];
                const double sq = (double)bar[pi].q, half = 0.5 * (sq - 1.0);
                const u64 m = A.mI[(size_t)sI * nt + t];
#pragma unroll
                for (int k = 0; k < NPAIR; ++k) {
                    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(rowAt(G.copy, pp, sI) + tileOff(k));
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const double yc = __longlong_as_double(h ? v.y : v.x);  // canonical
                        macc(a2[2 * k + h], (u64)yc, m);
                        neg[2 * k + h] += yc > half;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < NPAIR; ++k) {
                u64 o[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int w = 2 * k + h;
                    u64 out = subMultiple(sf_reduce128_acc(a2[w].lo, a2[w].hi, &CB), neg[w], A.sprod[t], CB);
                    if (rs) {
                        const double r = rr[w];
                        u64 lift = sf_reduce128((u64)(r < 0.0 ? r + qld : r), 0, &CB);
                        if (r < 0.0) lift = sf_sub(lift, A.lsub[t], CB.q);
                        out = sf_add(out, bmul(lift, A.pmod[t], CB), CB.q);
                    }
                    o[h] = out;
                }
                xr[k].x = o[0];
                xr[k].y = o[1];
            }
        }
        // the pass's twiddles for this prime, the tile -> LDS (as k_modup_col)
        const u64* gwI = tw + (size_t)pr * n;
        const u64* gwD = reinterpret_cast<const u64*>(twD) + (size_t)pr * n;
        const u64* gx = twS + (size_t)pr * n;
        if (!first) __syncthreads();  // the previous target's readers are done with s / tW
        first = false;
#pragma unroll
        for (int c = 0; c < kColPer; ++c) {
            const uint32_t e = threadIdx.x + c * NT;
            if (e < colTw) {
                tW[e] = fp ? gwD[e + 1] : gwI[e + 1];
                if (!fp) tX[e] = gx[e + 1];
            }
        }
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) {
            const uint32_t e = 2 * (threadIdx.x + k * NT);
            s[ldsSw(e)] = xr[k].x;
            s[ldsSw(e + 1)] = xr[k].y;
        }
        __syncthreads();
        if (fp) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                nttRoundFP<false, true, 2, 2, TILE, false, 8>(reinterpret_cast<double*>(s), T, 0u, 2 * r, qd[u],
                                                              reinterpret_cast<const double*>(tW), qi[u]);
                __syncthreads();
            }
        } else {
            for (uint32_t r = 0; r < 4; ++r) {
                nttRoundDyn<false, true, LE, TILE>(2, s, T, 0u, LE * r, q, tW, tX);
                __syncthreads();
            }
        }
        u64* out = rowAt(G.dst, pp, t);
#pragma unroll
        for (int k = 0; k < NPAIR; ++k) {
            const uint32_t e = 2 * (threadIdx.x + k * NT);
            ulonglong2 x;
            x.x = s[ldsSw(e)];
            x.y = s[ldsSw(e + 1)];
            if (fp) {
                x.x = d2u(fpReduce(__longlong_as_double(x.x), qd[u], qi[u]));
                x.y = d2u(fpReduce(__longlong_as_double(x.y), qd[u], qi[u]));
            }
            *reinterpret_cast<ulonglong2*>(out + tileOff(k)) = x;
        }
    }
}

// prims.h sfp_key_row on the device
__device__ __forceinline__ uint32_t keyRowOf(const sfp_key_geom& g, uint32_t p) {
    if (!g.rows) return p;
    return p < g.tail ? p : p < g.lq ? g.tail + (p - g.first) / g.world : g.pstart + (p - g.lq);
}

// key inner product over ext rows t < ell+K
// ext row t (prime primeOf(pm, t)) uses key row t < pm.split ? t : keyQ +
// (t - pm.split) of each digit's [b rows][a rows] block of keyRows rows, or
// the row of its prime when keyQ == SFP_KEY_ROW_BY_PRIME (sfp_key_row: a
// whole key, or this rank's slice of it).
struct KsInnerArgs {
    u64 *acc0, *acc1;
    const u64* ext;
    size_t extStride;
    const u64* key;
    uint32_t beta;
    sfp_limbs pm;
    uint32_t keyQ, keyRows;
    const u64 *fold0, *fold1;
    u64 foldK;
    int accum;
    const u64* pmul;
    sfp_key_geom kg;
    uint32_t gal;  // != 0: ext read through the automorphism X -> X^gal (sfp_ks_inner_aut)
};
template <int NG = 1>
__global__ __launch_bounds__(kThreads) void k_ks_inner(const ArgSet<KsInnerArgs, NG> S,
                                                       const sf_barrett* __restrict__ bar, uint32_t logn) {
    const KsInnerArgs& A = S.a[NG > 1 ? blockIdx.y : 0];
    u64* __restrict__ acc0 = A.acc0;
    u64* __restrict__ acc1 = A.acc1;
    const u64* __restrict__ ext = A.ext;
    const size_t extStride = A.extStride;
    const u64* __restrict__ key = A.key;
    const uint32_t beta = A.beta, keyQ = A.keyQ, keyRows = A.keyRows;
    const sfp_limbs pm = A.pm;
    const u64* __restrict__ fold0 = A.fold0;
    const u64* __restrict__ fold1 = A.fold1;
    const u64 foldK = A.foldK;
    const int accum = A.accum;
    const u64* __restrict__ pmul = A.pmul;
    const sfp_key_geom& kg = A.kg;
    // two coefficients per thread: 16-byte loads of every ext / key row
    const uint32_t ell = pm.split, NP = keyRows;
    const size_t pairs = ((size_t)pm.count << logn) >> 1;
    const uint32_t n = 1u << logn;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < pairs;
         i += (size_t)gridDim.x * kThreads) {
        const size_t e = 2 * i;
        const uint32_t t = (uint32_t)(e >> logn);
        const uint32_t x = (uint32_t)(e & (n - 1));
        const uint32_t pr = primeOf(pm, t);
        const uint32_t kr = keyQ == SFP_KEY_ROW_BY_PRIME ? keyRowOf(kg, pr) : (t < ell ? t : keyQ + (t - ell));
        const sf_barrett B = loadBar(bar, pr);
        Acc s0{0, 0}, s0b{0, 0}, s1{0, 0}, s1b{0, 0};
        // (gal: the two coefficients' sources, as k_automorph maps them)
        size_t src0 = e, src1 = e + 1;
        if (A.gal) {
            const u64 mask = 2ull * n - 1;
            const size_t row = e - x;
            src0 = row + sf_brev((uint32_t)((((2ull * sf_brev(x, logn) + 1) * A.gal & mask) - 1) >> 1), logn);
            src1 = row + sf_brev((uint32_t)((((2ull * sf_brev(x + 1, logn) + 1) * A.gal & mask) - 1) >> 1), logn);
        }
        for (uint32_t j = 0; j < beta; ++j) {
            ulonglong2 ev;
            if (A.gal) {
                ev.x = ext[j * extStride + src0];
                ev.y = ext[j * extStride + src1];
            } else {
                ev = *reinterpret_cast<const ulonglong2*>(ext + j * extStride + e);
            }
            const u64* kb = key + (size_t)j * 2 * NP * n + ((size_t)kr << logn) + x;
            const ulonglong2 b2 = *reinterpret_cast<const ulonglong2*>(kb);
            const ulonglong2 a2 = *reinterpret_cast<const ulonglong2*>(kb + (size_t)NP * n);
            macc(s0, ev.x, b2.x);
            macc(s0b, ev.y, b2.y);
            macc(s1, ev.x, a2.x);
            macc(s1b, ev.y, a2.y);
        }
        if (fold0 && t == ell - 1) {  // + P * d_l (sfp_ks_inner_fold)
            const ulonglong2 f0 = *reinterpret_cast<const ulonglong2*>(fold0 + e);
            const ulonglong2 f1 = *reinterpret_cast<const ulonglong2*>(fold1 + e);
            macc(s0, f0.x, foldK);
            macc(s0b, f0.y, foldK);
            macc(s1, f1.x, foldK);
            macc(s1b, f1.y, foldK);
        }
        ulonglong2 o0, o1;
        o0.x = sf_reduce128_acc(s0.lo, s0.hi, &B);
        o0.y = sf_reduce128_acc(s0b.lo, s0b.hi, &B);
        o1.x = sf_reduce128_acc(s1.lo, s1.hi, &B);
        o1.y = sf_reduce128_acc(s1b.lo, s1b.hi, &B);
        if (pmul) {  // sfp_ks_inner_mul: times a plaintext in the extended basis
            const ulonglong2 m = *reinterpret_cast<const ulonglong2*>(pmul + e);
            o0.x = bmul(o0.x, m.x, B);
            o0.y = bmul(o0.y, m.y, B);
            o1.x = bmul(o1.x, m.x, B);
            o1.y = bmul(o1.y, m.y, B);
        }
        if (accum) {  // sfp_ks_inner_acc: acc += the inner product
            const ulonglong2 p0 = *reinterpret_cast<const ulonglong2*>(acc0 + e);
            const ulonglong2 p1 = *reinterpret_cast<const ulonglong2*>(acc1 + e);
            o0.x = sf_add(o0.x, p0.x, B.q);
            o0.y = sf_add(o0.y, p0.y, B.q);
            o1.x = sf_add(o1.x, p1.x, B.q);
            o1.y = sf_add(o1.y, p1.y, B.q);
        }
        *reinterpret_cast<ulonglong2*>(acc0 + e) = o0;
        *reinterpret_cast<ulonglong2*>(acc1 + e) = o1;
    }
}

// ============================================================================
// sampling / loading

__device__ __forceinline__ u64 smix(u64 x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(kThreads) void k_uniform(u64* __restrict__ p, sfp_limbs m, u64 seed,
                                                      const sf_barrett* __restrict__ bar, uint32_t logn) {
    const size_t total = (size_t)m.count << logn;
    const uint32_t n = 1u << logn;
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < total;
         i += (size_t)gridDim.x * kThreads) {
        const uint32_t limb = (uint32_t)(i >> logn);
        const uint32_t pi = primeOf(m, limb);
        const sf_barrett B = loadBar(bar, pi);
        const u64 base = smix(seed ^ (0xD1B54A32D192ED03ULL * (u64)(pi + 1)));
        const u64 x = i & (n - 1);
        const u64 r0 = smix(base + 2 * x), r1 = smix(base + 2 * x + 1);
        p[i] = sf_reduce128_acc(r0, r1, &B);
    }
}

// One thread per coefficient: the signed input (pinned host memory, read
// once over the host link) is reduced into every limb.
__global__ __launch_bounds__(kThreads) void k_load_i64(u64* __restrict__ p, const int64_t* __restrict__ c,
                                                       sfp_limbs m, const sf_barrett* __restrict__ bar,
                                                       uint32_t logn) {
    const uint32_t n = 1u << logn;
    for (uint32_t x = blockIdx.x * kThreads + threadIdx.x; x < n; x += gridDim.x * kThreads) {
        const int64_t v = c[x];
        const u64 a = v < 0 ? (u64)(-(v + 1)) + 1 : (u64)v;
        for (uint32_t limb = 0; limb < m.count; ++limb) {
            const sf_barrett B = loadBar(bar, primeOf(m, limb));
            const u64 r = sf_reduce128(a, 0, &B);
            p[((size_t)limb << logn) + x] = (v < 0 && r) ? B.q - r : r;
        }
    }
}

// Plain copies run as kernels on the compute stream (never on the DMA
// engines), so every byte movement is ordered with the arithmetic around it.
__global__ __launch_bounds__(kThreads) void k_copy16(ulonglong2* __restrict__ dst,
                                                     const ulonglong2* __restrict__ src, size_t cnt) {
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < cnt; i += (size_t)gridDim.x * kThreads)
        dst[i] = src[i];
}
__global__ __launch_bounds__(kThreads) void k_copy1(unsigned char* __restrict__ dst,
                                                    const unsigned char* __restrict__ src, size_t cnt) {
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < cnt; i += (size_t)gridDim.x * kThreads)
        dst[i] = src[i];
}
__global__ __launch_bounds__(kThreads) void k_fill16(ulonglong2* __restrict__ dst, size_t cnt) {
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < cnt; i += (size_t)gridDim.x * kThreads)
        dst[i] = make_ulonglong2(0, 0);
}
__global__ __launch_bounds__(kThreads) void k_fill1(unsigned char* __restrict__ dst, size_t cnt) {
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < cnt; i += (size_t)gridDim.x * kThreads)
        dst[i] = 0;
}

// ============================================================================
// host side

// ============================================================================
// Stacked launches (sfp_stack_begin / sfp_stack_end)
//
// Inside a stacked region every lane's launches, event records and event
// waits are recorded per lane instead of issued.  stackFlush then issues them
// all on streams[0]: each lane's items in that lane's order, a wait only after
// the record it names, and -- whenever two lanes' next launches are the same
// kernel over different rows (the sort's two batches run the same op
// sequence, reference src/sort_algo.h:438-455, 713-742) -- those two as ONE
// launch whose grid holds the rows of both (ArgSet<T, 2>), or whose job table
// holds the jobs of both (conversions).  Per-row arithmetic is unchanged, so
// results are bit-identical; the sort issues about half the launches.
enum { STK_NONE = 0, STK_NTT = 1, STK_KS = 2, STK_CONV = 3, STK_MDRS = 4, STK_Y = 5 };

static uint64_t stkKey(const void* kern, uint32_t a, uint32_t b) {
    uint64_t h = 1469598103934665603ull;
    for (uint64_t x : {(uint64_t)(uintptr_t)kern, (uint64_t)a, (uint64_t)b}) h = (h ^ x) * 1099511628211ull;
    return h;
}

template <int NG>
using NttKernN = void (*)(RowGroupSet<NG>, const sf_barrett*, const u64*, const u64*, const u64*, const u64*,
                          uint32_t, const double*, const double*, const double*, const double*, int, const double*);
using NttKern2 = NttKernN<2>;
using NttKern4 = NttKernN<4>;
using NttKern8 = NttKernN<8>;
struct NttPay {
    RowGroup G;
    uint32_t rows;
    dim3 g;
    int threads, useFp;
    NttKern2 k2;
    NttKern4 k4;
    NttKern8 k8;
    const u64 *tw, *twS;
    const double *twD, *rowD;
};
template <int NG>
using KsKernN = void (*)(ArgSet<KsArgs, NG>, const sf_barrett*, const u64*, const u64*, uint32_t, const double*,
                         const double*, int, const double*);
struct KsPay {
    KsArgs a;
    uint32_t rows;
    dim3 g;
    int threads, useFp;
    KsKernN<2> k2;
    KsKernN<4> k4;
    KsKernN<8> k8;
};
using ConvKern = void (*)(ConvJobs, const sf_barrett*, const double*, uint32_t);
struct ConvPay {
    ConvJobs J;
    uint32_t njobs;
    dim3 g;
    ConvKern k;
};
struct MdrsPay {
    MdrsArgs M;  // (memset before filling: compared bytewise outside its jobs)
    dim3 g;
    ConvKern k;  // (same signature with MdrsArgs: stored through MdrsKern)
};
using MdrsKern = void (*)(MdrsArgs, const sf_barrett*, const double*, uint32_t);

// up to this many heads become one launch (the ArgSet<T, 4> kernels)
constexpr int kMergeMax = 8;

// The row-group kernels (k_ntt, k_ntt_ks): the heads' argument sets in one
// ArgSet<T, NG> (NG = 2 or 4), rows concatenated -- or alternating when every
// set has the same row count and fills the NG slots.
template <class T, int NG, class F>
static void launchSets(const T* const* a, const uint32_t* rows, int cnt, F&& launch) {
    ArgSet<T, NG> S;
    uint32_t total = 0;
    bool equal = true;
    for (int i = 0; i < NG; ++i) {
        S.a[i] = *a[std::min(i, cnt - 1)];
        S.start[i] = total;
        if (i < cnt) {
            total += rows[i];
            equal = equal && rows[i] == rows[0];
        }
    }
    S.inter = equal && cnt == NG;
    launch(S, total);
}

// grid.y arg-set kernels (k_ew, k_automorph, k_lin_wsum, k_ks_inner): the
// heads' sets with grid.y = their count (the largest grid.x; each set's
// grid-stride loop covers its own rows)
struct YPayBase {
    dim3 g;
    virtual ~YPayBase() = default;
    virtual void launchMany(sfp_dev* d, hipStream_t s, const YPayBase* const* h, int cnt) const = 0;
};
template <class Args>
struct YPay : YPayBase {
    Args a;
    void (*k2)(ArgSet<Args, 2>, const sf_barrett*, uint32_t);
    void (*k4)(ArgSet<Args, 4>, const sf_barrett*, uint32_t);
    template <int NG, class K>
    void go(sfp_dev* d, hipStream_t s, const YPayBase* const* h, int cnt, K k) const {
        ArgSet<Args, NG> S;
        uint32_t gx = 0;
        for (int i = 0; i < NG; ++i) {
            const auto& o = static_cast<const YPay<Args>&>(*h[std::min(i, cnt - 1)]);
            S.a[i] = o.a;
            S.start[i] = 0;
            gx = std::max(gx, o.g.x);
        }
        S.inter = 0;
        hipLaunchKernelGGL(k, dim3(gx, cnt), dim3(kThreads), 0, s, S, d->bar, d->logn);
    }
    void launchMany(sfp_dev* d, hipStream_t s, const YPayBase* const* h, int cnt) const override {
        if (cnt == 2)
            go<2>(d, s, h, cnt, k2);
        else
            go<4>(d, s, h, cnt, k4);
    }
};
template <class Args>
static void issueY(sfp_dev* d, void (*k1)(ArgSet<Args, 1>, const sf_barrett*, uint32_t),
                   void (*k2)(ArgSet<Args, 2>, const sf_barrett*, uint32_t),
                   void (*k4)(ArgSet<Args, 4>, const sf_barrett*, uint32_t), dim3 g, const Args& a) {
    ArgSet<Args, 1> S;
    S.a[0] = a;
    S.start[0] = 0;
    S.inter = 0;
    StackRec r;
    r.go = [=](hipStream_t s_) { hipLaunchKernelGGL(k1, g, dim3(kThreads), 0, s_, S, d->bar, d->logn); };
    if (d->stackOn) {
        auto P = std::make_shared<YPay<Args>>();
        P->a = a;
        P->k2 = k2;
        P->k4 = k4;
        P->g = g;
        r.cls = STK_Y;
        r.key = stkKey((const void*)k1, 0, 0);
        r.pay = std::move(P);
    }
    issueRec(d, std::move(r));
}

// Issue the heads h[0..cnt) (2 <= cnt <= kMergeMax, one class and key) as one
// launch on s; false if their arguments cannot share one (the caller then
// issues them apart); check: only report whether they can.
static bool stackMerge(sfp_dev* d, const StackRec* const* h, int cnt, hipStream_t s, bool check) {
    auto pay = [&](int i) { return h[i]->pay.get(); };
    switch (h[0]->cls) {
        case STK_NTT: {
            const NttPay* P[kMergeMax];
            const RowGroup* G[kMergeMax];
            uint32_t rows[kMergeMax], total = 0;
            for (int i = 0; i < cnt; ++i) {
                P[i] = static_cast<const NttPay*>(pay(i));
                G[i] = &P[i]->G;
                rows[i] = P[i]->rows;
                total += rows[i];
                if (P[i]->g.x != P[0]->g.x || P[i]->useFp != P[0]->useFp) return false;
            }
            if (total > 65535u || !(cnt == 2 ? (bool)P[0]->k2 : cnt <= 4 ? (bool)P[0]->k4 : (bool)P[0]->k8))
                return false;
            if (check) return true;
            const NttPay& A = *P[0];
            auto launch = [&](const auto& S, uint32_t tot) {
                using SetT = std::decay_t<decltype(S)>;
                constexpr int NG = sizeof(SetT::a) / sizeof(RowGroup);
                NttKernN<NG> k;
                if constexpr (NG == 2)
                    k = A.k2;
                else if constexpr (NG == 4)
                    k = A.k4;
                else
                    k = A.k8;
                hipLaunchKernelGGL(k, dim3(A.g.x, tot), dim3(A.threads), 0, s, S, d->bar, A.tw, A.twS, d->ninv,
                                   d->ninvS, d->logn, A.twD, d->qinvD, d->ninvD, d->ninvQ, A.useFp, A.rowD);
            };
            if (cnt == 2)
                launchSets<RowGroup, 2>(G, rows, cnt, launch);
            else if (cnt <= 4)
                launchSets<RowGroup, 4>(G, rows, cnt, launch);
            else
                launchSets<RowGroup, 8>(G, rows, cnt, launch);
            return true;
        }
        case STK_KS: {
            const KsPay* P[kMergeMax];
            const KsArgs* A[kMergeMax];
            uint32_t rows[kMergeMax], total = 0;
            for (int i = 0; i < cnt; ++i) {
                P[i] = static_cast<const KsPay*>(pay(i));
                A[i] = &P[i]->a;
                rows[i] = P[i]->rows;
                total += rows[i];
                if (P[i]->g.x != P[0]->g.x || P[i]->useFp != P[0]->useFp) return false;
            }
            if (total > 65535u || !(cnt == 2 ? (bool)P[0]->k2 : cnt <= 4 ? (bool)P[0]->k4 : (bool)P[0]->k8))
                return false;
            if (check) return true;
            const KsPay& B = *P[0];
            auto launch = [&](const auto& S, uint32_t tot) {
                using SetT = std::decay_t<decltype(S)>;
                constexpr int NG = sizeof(SetT::a) / sizeof(KsArgs);
                KsKernN<NG> k;
                if constexpr (NG == 2)
                    k = B.k2;
                else if constexpr (NG == 4)
                    k = B.k4;
                else
                    k = B.k8;
                hipLaunchKernelGGL(k, dim3(B.g.x, tot), dim3(B.threads), 0, s, S, d->bar, d->psi, d->psiS, d->logn,
                                   d->psiD, d->qinvD, B.useFp, d->rowD);
            };
            if (cnt == 2)
                launchSets<KsArgs, 2>(A, rows, cnt, launch);
            else if (cnt <= 4)
                launchSets<KsArgs, 4>(A, rows, cnt, launch);
            else
                launchSets<KsArgs, 8>(A, rows, cnt, launch);
            return true;
        }
        case STK_CONV: {
            const ConvPay* P[kMergeMax];
            uint32_t jobs = 0, gz = 0;
            for (int i = 0; i < cnt; ++i) {
                P[i] = static_cast<const ConvPay*>(pay(i));
                if (P[i]->k != P[0]->k || P[i]->g.x != P[0]->g.x) return false;
                jobs += P[i]->njobs;
                gz = std::max(gz, P[i]->g.z);
            }
            if (jobs > (uint32_t)kMaxConvJobs) return false;
            if (check) return true;
            ConvJobs J;
            uint32_t at = 0;
            for (int i = 0; i < cnt; ++i)
                for (uint32_t k = 0; k < P[i]->njobs; ++k) J.j[at++] = P[i]->J.j[k];
            hipLaunchKernelGGL(P[0]->k, dim3(P[0]->g.x, jobs, gz), dim3(kThreads), 0, s, J, d->bar, d->qinvD,
                               d->logn);
            return true;
        }
        case STK_MDRS: {
            const MdrsPay* P[kMergeMax];
            uint32_t jobs = 0;
            MdrsArgs x0 = static_cast<const MdrsPay*>(pay(0))->M;
            std::memset(x0.j, 0, sizeof x0.j);
            for (int i = 0; i < cnt; ++i) {
                P[i] = static_cast<const MdrsPay*>(pay(i));
                if (P[i]->k != P[0]->k || P[i]->g.x != P[0]->g.x || P[i]->g.z != P[0]->g.z) return false;
                MdrsArgs x = P[i]->M;
                std::memset(x.j, 0, sizeof x.j);
                if (std::memcmp(&x, &x0, sizeof x)) return false;  // another table / level
                jobs += P[i]->g.y;
            }
            if (jobs > (uint32_t)kMdrsJobs) return false;
            if (check) return true;
            MdrsArgs M = P[0]->M;
            uint32_t at = 0;
            for (int i = 0; i < cnt; ++i)
                for (uint32_t k = 0; k < P[i]->g.y; ++k) M.j[at++] = P[i]->M.j[k];
            hipLaunchKernelGGL(reinterpret_cast<MdrsKern>(P[0]->k), dim3(P[0]->g.x, jobs, P[0]->g.z), dim3(kThreads),
                               0, s, M, d->bar, d->qinvD, d->logn);
            return true;
        }
        case STK_Y: {
            if (cnt > 4) return false;  // (four element-wise argument sets fill the 4 KB of kernel arguments)
            if (check) return true;
            const YPayBase* Y[kMergeMax];
            for (int i = 0; i < cnt; ++i) Y[i] = static_cast<const YPayBase*>(pay(i));
            Y[0]->launchMany(d, s, Y, cnt);
            return true;
        }
        default:
            return false;
    }
}

// Issue one launch (or a merged pair) on s, bracketed by HIP events when its
// family is being timed (sfp_prof_set) and this launch is a sampled one.
template <class F>
static void stackTimed(sfp_dev* d, hipStream_t s, uint32_t fam, double bytes, F&& go) {
    if (fam >= SFP_FAM_COUNT || d->capture) return go();
    sfp_dev::ProfFam& f = d->prof[fam];
    if (!f.period || (f.seen++ % f.period) != 0) return go();
    hipEvent_t a = takeEvent(d), b = takeEvent(d);
    SFP_CHECK(hipEventRecord(a, s));
    go();
    SFP_CHECK(hipEventRecord(b, s));
    f.pending.push_back({a, b});
    f.timed++;
    f.bytes += bytes;
    if (f.pending.size() >= 8192) profFlush(d, f);
}

static void stackFlush(sfp_dev* d) {
    if (!d->stackOn) return;
    const hipStream_t s = d->stackStream ? d->stackStream : d->streams[0];
    constexpr int L = SFP_MAX_LANES;
    size_t at[L] = {};
    std::unordered_set<uint64_t> done;  // records issued so far
    auto left = [&](int l) { return d->stack[l].size() - at[l]; };
    auto head = [&](int l) -> StackRec& { return d->stack[l][at[l]]; };
    auto blocked = [&](int l) {
        const StackRec& r = head(l);
        return r.kind == StackRec::EV_WAIT && r.id && !done.count(r.id);
    };
    for (;;) {
        // records and satisfied waits first: they cost nothing and unblock
        for (bool moved = true; moved;) {
            moved = false;
            for (int l = 0; l < L; ++l)
                while (left(l) && head(l).kind != StackRec::LAUNCH && !blocked(l)) {
                    const StackRec& r = head(l);
                    if (r.kind == StackRec::EV_RECORD) {
                        SFP_CHECK(hipEventRecord(r.ev->e, s));
                        done.insert(r.id);
                    } else if (!r.id) {  // an event recorded before the region
                        SFP_CHECK(hipStreamWaitEvent(s, r.ev->e, 0));
                    }  // (a record issued above: same stream, already ordered)
                    ++at[l];
                    moved = true;
                }
        }
        int cand[L], nc = 0;
        for (int l = 0; l < L; ++l)
            if (left(l) && head(l).kind == StackRec::LAUNCH) cand[nc++] = l;
        if (!nc) {
            for (int l = 0; l < L; ++l)
                if (left(l)) {  // a wait whose record never comes: issue the rest in lane order
                    record(d, "stacked region: an event wait without its record", hipErrorInvalidValue);
                    for (int k = 0; k < L; ++k)
                        for (; left(k); ++at[k])
                            if (head(k).kind == StackRec::LAUNCH) head(k).go(s);
                    break;
                }
            break;
        }
        // the largest group of heads of one class and key (up to kMergeMax,
        // lanes furthest behind first) becomes one launch
        int best[kMergeMax], nb = 0;
        for (int i = 0; i < nc; ++i) {
            const StackRec& a = head(cand[i]);
            if (!a.cls) continue;
            int grp[kMergeMax], ng = 0;
            for (int j = i; j < nc && ng < kMergeMax; ++j) {
                const StackRec& b = head(cand[j]);
                if (b.cls == a.cls && b.key == a.key) grp[ng++] = cand[j];
            }
            if (ng > nb) {
                nb = ng;
                std::copy(grp, grp + ng, best);
            }
        }
        while (nb >= 2) {
            const StackRec* hs[kMergeMax];
            double bytes = 0;
            for (int i = 0; i < nb; ++i) {
                hs[i] = &head(best[i]);
                bytes += hs[i]->bytes;
            }
            if (stackMerge(d, hs, nb, s, true)) {
                stackTimed(d, s, hs[0]->fam, bytes, [&] { stackMerge(d, hs, nb, s, false); });
                for (int i = 0; i < nb; ++i) ++at[best[i]];
                ++d->stkMerged;
                break;
            }
            --nb;  // (a group whose arguments do not fit one launch: try fewer)
        }
        if (nb >= 2) continue;
        // alone: the lane furthest behind (most items left) goes first, which
        // realigns lanes whose sequences differ by an op (batch 0's offset)
        int one = cand[0];
        for (int i = 1; i < nc; ++i)
            if (left(cand[i]) > left(one)) one = cand[i];
        const StackRec& r = head(one);
        stackTimed(d, s, r.fam, r.bytes, [&] { r.go(s); });
        ++at[one];
        ++d->stkSingle;
    }
    for (int l = 0; l < L; ++l) d->stack[l].clear();
    std::lock_guard<std::mutex> g(d->evMu);
    for (sfp_event* e : d->stackFreedEv) d->evFree.push_back(e);
    d->stackFreedEv.clear();
}

static unsigned ewGrid(size_t work) {
    size_t g = (work + kThreads - 1) / kThreads;
    if (g > 256 * 16) g = 256 * 16;
    return (unsigned)(g ? g : 1);
}

// Device-side byte copy on the compute stream (either side may be pinned
// host memory).  Never uses the DMA engines: see DESIGN.md "transfers".
// SFHE_DMA_COPY=1 (experiment): the same copies as
// hipMemcpyAsync on the compute stream (the SDMA engines), ordered like every
// other prim of the lane.
static bool dmaCopy() {
    static const bool on = [] {
        const char* v = std::getenv("SFHE_DMA_COPY");
        return v && *v == '1';
    }();
    return on;
}

// immediate: issued on the stream now even inside a stacked region (host
// uploads and downloads through the ring / bounce buffers: the deferred
// launches that read an upload are issued after it on the same stream)
static void devCopy(sfp_dev* d, void* dst, const void* src, size_t b, bool immediate = false) {
    if (!b) return;
    if (dmaCopy()) {
        if (immediate || !d->stackOn)
            SFP_CHECK(hipMemcpyAsync(dst, src, b, hipMemcpyDefault, d->st()));
        else
            issue(d, [=](hipStream_t s_) { hipMemcpyAsync(dst, src, b, hipMemcpyDefault, s_); });
        return;
    }
    std::function<void(hipStream_t)> go;
    if ((((uintptr_t)dst | (uintptr_t)src | b) & 15) == 0) {
        const size_t cnt = b / 16;
        go = [=](hipStream_t s_) {
            hipLaunchKernelGGL(k_copy16, dim3(ewGrid(cnt)), dim3(kThreads), 0, s_, (ulonglong2*)dst,
                               (const ulonglong2*)src, cnt);
        };
    } else {
        go = [=](hipStream_t s_) {
            hipLaunchKernelGGL(k_copy1, dim3(ewGrid(b)), dim3(kThreads), 0, s_, (unsigned char*)dst,
                               (const unsigned char*)src, b);
        };
    }
    if (immediate)
        go(d->st());
    else
        issue(d, std::move(go));
    checkLaunch(d, "copy");
}

static void devZero(sfp_dev* d, void* dst, size_t b) {
    if (!b) return;
    if ((((uintptr_t)dst | b) & 15) == 0) {
        SFP_GO(k_fill16, dim3(ewGrid(b / 16)), dim3(kThreads), (ulonglong2*)dst, b / 16);
    } else {
        SFP_GO(k_fill1, dim3(ewGrid(b)), dim3(kThreads), (unsigned char*)dst, b);
    }
    checkLaunch(d, "zero");
}

// Small host array -> device memory, ordered on the stream: staged in the
// pinned ring, pulled across by a copy kernel.  The ring region is reused
// only after the stream has drained past every earlier pull.
// Copy of a small host array in the open capture's arena (device address;
// the arena is uploaded when the capture ends).
static const u64* arenaPut(sfp_dev* d, const void* src, size_t bytes) {
    sfp_graph* g = d->capture;
    const size_t words = ((bytes + 255) & ~(size_t)255) / 8;
    if (g->arena.empty() || g->arena.back().used + words > g->arena.back().host.size()) {
        GraphChunk c;
        const size_t cap = std::max(words, (size_t)1 << 19);  // 4 MiB chunks
        if (hipMalloc((void**)&c.dev, cap * 8) != hipSuccess) {
            hipGetLastError();
            captureFail(d, "graph arena allocation");
            return nullptr;
        }
        c.host.assign(cap, 0);
        g->arena.push_back(std::move(c));
    }
    GraphChunk& c = g->arena.back();
    std::memcpy(c.host.data() + c.used, src, bytes);
    const u64* dv = c.dev + c.used;
    c.used += words;
    return dv;
}

// Host bytes -> device address dst through the pinned ring, ordered on the
// current lane (ringPut's rules: the region is reused after a full drain).
static void ringUpload(sfp_dev* d, void* dst, const void* src, size_t bytes) {
    const size_t span = (bytes + 255) & ~(size_t)255;
    if (span > d->ringCap) return record(d, "argument ring: upload larger than the ring", hipErrorInvalidValue);
    if (d->ringOff + span > d->ringCap) {
        syncAll(d);
        d->ringOff = 0;
    }
    char* h = d->hring + d->ringOff;
    std::memcpy(h, src, bytes);
    devCopy(d, dst, h, bytes, true);
    d->ringOff += span;
}

static void constClear(sfp_dev* d) {
    for (auto& kv : d->cmap)
        for (auto& e : kv.second)
            if (e.ev) hipEventDestroy(e.ev);
    d->cmap.clear();
}

static void* ringPut(sfp_dev* d, const void* src, size_t bytes) {
    if (d->capture) return const_cast<u64*>(arenaPut(d, src, bytes));
    const size_t span = (bytes + 255) & ~(size_t)255;  // keep entries 256-B aligned
    if (span > d->ringCap) {  // (would write past the pinned ring) -- callers chunk their uploads
        record(d, "argument ring: upload larger than the ring", hipErrorInvalidValue);
        return nullptr;
    }
    if (d->ringOff + span > d->ringCap) {
        syncAll(d);
        d->ringOff = 0;
    }
    char* h = d->hring + d->ringOff;
    char* dv = d->dring + d->ringOff;
    std::memcpy(h, src, bytes);  // only the caller's bytes: src may end right there
    devCopy(d, dv, h, bytes, true);
    d->ringOff += span;
    return dv;
}

// Bulk host -> device through the bounce buffer, chunk by chunk.
static void hostToDev(sfp_dev* d, void* dst, const void* src, size_t b) {
    if (d->capture) return captureFail(d, "host-to-device upload inside the captured region");
    syncAll(d);  // the bounce buffer is shared by every lane
    for (size_t off = 0; off < b; off += d->bounceCap) {
        const size_t c = b - off < d->bounceCap ? b - off : d->bounceCap;
        std::memcpy(d->bounce, (const char*)src + off, c);
        devCopy(d, (char*)dst + off, d->bounce, c, true);
        SFP_CHECK(hipStreamSynchronize(d->st()));
    }
}

static void devToHost(sfp_dev* d, void* dst, const void* src, size_t b) {
    if (d->capture) return captureFail(d, "device-to-host download inside the captured region");
    syncAll(d);
    for (size_t off = 0; off < b; off += d->bounceCap) {
        const size_t c = b - off < d->bounceCap ? b - off : d->bounceCap;
        devCopy(d, d->bounce, (const char*)src + off, c, true);
        SFP_CHECK(hipStreamSynchronize(d->st()));
        std::memcpy((char*)dst + off, d->bounce, c);
    }
}

// Device copy of a small constant array, shared by every call with the same
// contents (uploaded once; the stream is drained only on a miss).
static const u64* devConst(sfp_dev* d, const u64* v, size_t count) {
    uint64_t h = 1469598103934665603ull ^ count;
    for (size_t i = 0; i < count; ++i) h = (h ^ v[i]) * 1099511628211ull;
    if (d->capture) {  // the graph's own immutable copy (the pool's generations retire)
        auto& b = d->capture->consts[h];
        for (auto& e : b)
            if (e.first.size() == count && std::equal(v, v + count, e.first.begin())) return e.second;
        const u64* p = arenaPut(d, v, count * 8);
        if (p) b.push_back({std::vector<u64>(v, v + count), p});
        return p;
    }
    auto& bucket = d->cmap[h];
    for (auto& e : bucket)
        if (e.v.size() == count && std::equal(v, v + count, e.v.begin())) {
            if (e.ev && e.lane != d->cur) {  // uploaded on another lane: order after it
                SFP_CHECK(hipStreamWaitEvent(d->st(), e.ev, 0));
                if (hipEventQuery(e.ev) == hipSuccess) {  // done: later hits need no wait
                    hipEventDestroy(e.ev);
                    e.ev = nullptr;
                }
            }
            return d->cpool + e.off;
        }
    const size_t words = (count + 1) & ~(size_t)1;  // keep 16-B alignment
    if (!d->cpool || d->cpoolOff + words > d->cpoolCap) {
        // Two generations: the full pool is retired, not overwritten, so
        // pointers a prim obtained just before this call (for the same
        // launch) stay valid; the generation before it is free once every
        // queued kernel has drained.
        syncAll(d);
        if (!d->cpoolOld) {
            d->cpoolCap = (size_t)1 << 19;  // 4 MiB per generation
            SFP_CHECK(hipMalloc((void**)&d->cpoolOld, d->cpoolCap * 8));
        }
        std::swap(d->cpool, d->cpoolOld);
        if (!d->cpool) SFP_CHECK(hipMalloc((void**)&d->cpool, d->cpoolCap * 8));
        constClear(d);
        d->cpoolOff = 0;
    }
    const size_t off = d->cpoolOff;
    d->cpoolOff += words;
    // through the pinned ring on this lane's stream: a miss no longer drains
    // the device (the cold sort's first use of every per-level constant)
    ringUpload(d, d->cpool + off, v, count * 8);
    hipEvent_t ev = nullptr;
    if (d->nLanes > 1 && !d->serial) {
        SFP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        SFP_CHECK(hipEventRecord(ev, d->st()));
    }
    d->cmap[h].push_back({std::vector<u64>(v, v + count), off, d->cur, ev});
    return d->cpool + off;
}

// (C linkage comes from the declarations in prims.h)

const char* sfp_backend_name(void) { return "hip-gfx950"; }

sfp_dev* sfp_create(int device, const sfp_tables* t) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    auto* d = new sfp_dev;
    d->device = device;
    d->logn = t->logn;
    d->n = 1u << t->logn;
    d->np = t->nprimes;
    if (d->logn < 10 || d->logn > 17) {
        delete d;
        // rings 2^10 .. 2^17: up to 2^11 the NTT runs k_ntt_small; the COL
        // pass stages 2^logR - 1 <= kNttColTw twiddles in LDS (logR <= 9)
        return nullptr;
    }
    d->nLanes = 4;
    if (const char* v = std::getenv("SFHE_LANES"))
        d->nLanes = std::max(1, std::min(SFP_MAX_LANES - SFP_BATCH_MAX, std::atoi(v)));
    for (int l = 0; l < d->nLanes; ++l)
        if (hipStreamCreateWithFlags(&d->streams[l], hipStreamNonBlocking) != hipSuccess) {
            for (int k = 0; k < l; ++k) hipStreamDestroy(d->streams[k]);
            delete d;
            return nullptr;
        }
    d->hbar.resize(d->np);
    for (uint32_t i = 0; i < d->np; ++i) d->hbar[i] = sf_make_barrett(t->primes[i]);
    const size_t tn = (size_t)d->np * d->n * 8;
    bool ok = hipMalloc(&d->bar, d->np * sizeof(sf_barrett)) == hipSuccess &&
              hipMalloc(&d->psi, tn) == hipSuccess && hipMalloc(&d->psiS, tn) == hipSuccess &&
              hipMalloc(&d->ipsi, tn) == hipSuccess && hipMalloc(&d->ipsiS, tn) == hipSuccess &&
              hipMalloc(&d->ninv, d->np * 8) == hipSuccess &&
              hipMalloc(&d->ninvS, d->np * 8) == hipSuccess && hipMalloc(&d->psiD, tn) == hipSuccess &&
              hipMalloc(&d->ipsiD, tn) == hipSuccess && hipMalloc(&d->rowD, (size_t)d->np * 8 * (d->n >> 8) * 8) == hipSuccess &&
              hipMalloc(&d->irowD, (size_t)d->np * 8 * (d->n >> 8) * 8) == hipSuccess &&
              hipMalloc(&d->qinvD, d->np * 8) == hipSuccess &&
              hipMalloc(&d->ninvD, d->np * 8) == hipSuccess && hipMalloc(&d->ninvQ, d->np * 8) == hipSuccess;
    d->ringCap = (size_t)16 << 20;
    if (const char* v = std::getenv("SFHE_ARG_RING_MB"))  // (tests: force chunked uploads)
        d->ringCap = (size_t)std::max(1, std::atoi(v)) << 20;
    d->bounceCap = (size_t)32 << 20;
    ok = ok &&
         hipHostMalloc((void**)&d->hring, d->ringCap, hipHostMallocMapped | hipHostMallocCoherent) ==
             hipSuccess &&
         hipMalloc((void**)&d->dring, d->ringCap) == hipSuccess &&
         hipHostMalloc((void**)&d->bounce, d->bounceCap, hipHostMallocMapped | hipHostMallocCoherent) ==
             hipSuccess;
    if (!ok) {
        delete d;
        return nullptr;
    }
    hostToDev(d, d->bar, d->hbar.data(), d->np * sizeof(sf_barrett));
    hostToDev(d, d->psi, t->psi_rev, tn);
    hostToDev(d, d->psiS, t->psi_rev_shoup, tn);
    hostToDev(d, d->ipsi, t->ipsi_rev, tn);
    hostToDev(d, d->ipsiS, t->ipsi_rev_shoup, tn);
    hostToDev(d, d->ninv, t->n_inv, d->np * 8);
    d->hninv.assign(t->n_inv, t->n_inv + d->np);
    hostToDev(d, d->ninvS, t->n_inv_shoup, d->np * 8);
    {
        // FP64 twiddle values (the kernels form W/q in registers)
        std::vector<double> a((size_t)d->np * d->n), qi(d->np), ni(d->np), nq(d->np);
        auto fill = [&](const uint64_t* tab, double* A) {
            for (size_t o = 0; o < (size_t)d->np * d->n; ++o) A[o] = (double)tab[o];
        };
        fill(t->psi_rev, a.data());
        hostToDev(d, d->psiD, a.data(), tn);
        fill(t->ipsi_rev, a.data());
        hostToDev(d, d->ipsiD, a.data(), tn);
        // ROW-pass row factors (rowTwIssue): psi_rev[row << k] per prime, k < 8, row < n / 256
        const uint32_t R = d->n >> 8;
        std::vector<double> rf((size_t)d->np * 8 * R), irf((size_t)d->np * 8 * R);
        for (uint32_t p = 0; p < d->np; ++p)
            for (uint32_t k = 0; k < 8; ++k)
                for (uint32_t row = 0; row < R; ++row) {
                    const size_t o = ((size_t)p * 8 + k) * R + row, src = (size_t)p * d->n + ((size_t)row << k);
                    rf[o] = (double)t->psi_rev[src];
                    irf[o] = (double)t->ipsi_rev[src];
                }
        hostToDev(d, d->rowD, rf.data(), rf.size() * 8);
        hostToDev(d, d->irowD, irf.data(), irf.size() * 8);
        for (uint32_t p = 0; p < d->np; ++p) {
            const double q = (double)d->hbar[p].q;
            qi[p] = 1.0 / q;
            ni[p] = (double)t->n_inv[p];
            nq[p] = (double)t->n_inv[p] / q;
        }
        hostToDev(d, d->qinvD, qi.data(), d->np * 8);
        hostToDev(d, d->ninvD, ni.data(), d->np * 8);
        hostToDev(d, d->ninvQ, nq.data(), d->np * 8);
    }
    if (!d->err.empty()) {
        sfp_destroy(d);
        return nullptr;
    }
    return d;
}

// RCCL is opened on first use (dlopen), not linked: processes that never
// shard do not load it, and its threads and teardown stay out of them.
struct RcclApi {
    bool ok = false;
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*errorString)(ncclResult_t) = nullptr;
};

static RcclApi& rcclApi() {
    static RcclApi a;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) return;
        auto sym = [h](auto& f, const char* n) { f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, n)); };
        sym(a.getUniqueId, "ncclGetUniqueId");
        sym(a.commInitRank, "ncclCommInitRank");
        sym(a.commDestroy, "ncclCommDestroy");
        sym(a.allGather, "ncclAllGather");
        sym(a.broadcast, "ncclBroadcast");
        sym(a.errorString, "ncclGetErrorString");
        a.ok = a.getUniqueId && a.commInitRank && a.commDestroy && a.allGather && a.broadcast && a.errorString;
    });
    return a;
}

void sfp_destroy(sfp_dev* d) {
    if (!d) return;
    syncAll(d);
    for (auto& kv : d->plans)
        if (kv.second) freePlan(kv.second);
    d->plans.clear();
    if (d->nccl) rcclApi().commDestroy(d->nccl);
    if (d->gnccl) rcclApi().commDestroy(d->gnccl);
    for (sfp_event* e : d->evFree) {
        hipEventDestroy(e->e);
        delete e;
    }
    for (auto& f : d->prof) profFlush(d, f);
    for (hipEvent_t e : d->evPool) hipEventDestroy(e);
    constClear(d);
    hipFree(d->bar);
    hipFree(d->psi);
    hipFree(d->psiS);
    hipFree(d->ipsi);
    hipFree(d->ipsiS);
    hipFree(d->ninv);
    hipFree(d->ninvS);
    for (double* x : {d->psiD, d->ipsiD, d->rowD, d->irowD, d->qinvD, d->ninvD, d->ninvQ}) hipFree(x);
    hipFree(d->dring);
    hipHostFree(d->hring);
    hipHostFree(d->bounce);
    hipFree(d->cpool);
    hipFree(d->cpoolOld);
    hipFree(d->encRot);
    hipFree(d->encKsi);
    for (u64* p : d->scr) hipFree(p);
    for (void* p : d->retired) hipFree(p);
    for (int l = 0; l < d->nLanes; ++l) hipStreamDestroy(d->streams[l]);
    delete d;
}

void* sfp_alloc(sfp_dev* d, size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 8) != hipSuccess) {
        hipGetLastError();
        return nullptr;
    }
    return p;
}
void sfp_free(sfp_dev* d, void* p) {
    (void)d;
    hipFree(p);
}
void sfp_h2d(sfp_dev* d, void* dst, const void* src, size_t b) { hostToDev(d, dst, src, b); }
void sfp_d2h(sfp_dev* d, void* dst, const void* src, size_t b) { devToHost(d, dst, src, b); }
void sfp_d2d(sfp_dev* d, void* dst, const void* src, size_t b) { devCopy(d, dst, src, b); }
void sfp_zero(sfp_dev* d, void* dst, size_t b) { devZero(d, dst, b); }
void sfp_sync(sfp_dev* d) { syncAll(d); }

int sfp_lanes(sfp_dev* d) { return d->nLanes; }
void sfp_set_lane(sfp_dev* d, int lane) {
    if (lane < 0 || lane >= d->nLanes) {
        record(d, "set_lane", hipErrorInvalidValue);
        return;
    }
    if (d->batchOn) {  // a batched op's lane stays its virtual lane
        if (lane != d->batchCur) record(d, "set_lane (inside a batch)", hipErrorInvalidValue);
    } else {
        d->cur = lane;
    }
    // HIP's current device is per host thread; a lane may be driven from a
    // thread other than the one that created the device
    thread_local int curDev = -1;
    if (curDev != d->device) {
        SFP_CHECK(hipSetDevice(d->device));
        curDev = d->device;
    }
}
int sfp_get_lane(sfp_dev* d) { return d->cur; }

sfp_event* sfp_event_record(sfp_dev* d) {
    sfp_event* e = nullptr;
    {
        std::lock_guard<std::mutex> g(d->evMu);
        if (!d->evFree.empty()) {
            e = d->evFree.back();
            d->evFree.pop_back();
        }
    }
    if (!e) {
        e = new sfp_event;
        SFP_CHECK(hipEventCreateWithFlags(&e->e, hipEventDisableTiming));
    }
    e->lane = d->cur;
    if (d->stackOn) {  // recorded at its place in the lane's sequence by stackFlush
        StackRec r;
        r.kind = StackRec::EV_RECORD;
        r.ev = e;
        r.id = e->recId = ++d->recSeq;
        d->stack[d->cur].push_back(std::move(r));
        return e;
    }
    e->recId = 0;
    SFP_CHECK(hipEventRecord(e->e, d->st()));
    return e;
}
void sfp_event_wait(sfp_dev* d, const sfp_event* e) {
    if (!e || e->lane == d->cur) return;
    if (d->stackOn) {
        StackRec r;
        r.kind = StackRec::EV_WAIT;
        r.ev = const_cast<sfp_event*>(e);
        r.id = e->recId;  // 0: a record made before the region (a real event already)
        d->stack[d->cur].push_back(std::move(r));
        return;
    }
    SFP_CHECK(hipStreamWaitEvent(d->st(), e->e, 0));
}
int sfp_event_done(sfp_dev* d, const sfp_event* e) {
    // a capture starts after every lane drained: earlier events are complete
    if (d->capture) return 1;
    stackFlush(d);
    return !e || hipEventQuery(e->e) == hipSuccess;
}
void sfp_event_free(sfp_dev* d, sfp_event* e) {
    if (!e) return;
    std::lock_guard<std::mutex> g(d->evMu);
    // inside a stacked region a deferred record or wait may still name it:
    // reusable only after the flush
    if (d->stackOn && e->recId) return d->stackFreedEv.push_back(e);
    d->evFree.push_back(e);  // re-recording later is safe: waits bind at enqueue time
}

void sfp_stack_begin(sfp_dev* d) {
    if (d->stackOn) return;
    d->stackStream = nullptr;  // (lanes: the flush issues on lane 0)
    static const bool on = [] {
        const char* v = std::getenv("SFHE_STACK");
        return !v || *v != '0';
    }();
    if (!on) return;
    d->stackOn = true;
}
void sfp_stack_end(sfp_dev* d) {
    if (d->batchOn) return;  // (a batched op's region ends with sfp_batch_end)
    stackFlush(d);
    d->stackOn = false;
}

// Batched ops: `count` (<= SFP_BATCH_MAX) independent ops issued one after the
// other by the host, each after sfp_batch_lane(i), are recorded on virtual
// lanes and issued at sfp_batch_end on the caller's stream, identical
// launches of the ops merged (up to kMergeMax into one).  Inside a stacked
// lane region (no nesting) the ops run as issued.
int sfp_batch_begin(sfp_dev* d, uint32_t count) {
    static const bool on = [] {
        const char* v = std::getenv("SFHE_BATCH");
        return !v || *v != '0';
    }();
    if (!on || d->stackOn || count < 2 || count > SFP_BATCH_MAX ||
        d->nLanes > SFP_MAX_LANES - SFP_BATCH_MAX)
        return 0;
    d->stackStream = d->st();
    d->batchCur = d->cur;
    d->batchOn = true;
    d->stackOn = true;
    return 1;
}
void sfp_batch_lane(sfp_dev* d, uint32_t i) {
    if (d->batchOn) d->cur = (int)(SFP_MAX_LANES - SFP_BATCH_MAX + i);  // (its own list and scratch)
}
void sfp_batch_end(sfp_dev* d) {
    if (!d->batchOn) return;
    d->cur = d->batchCur;
    stackFlush(d);
    d->batchOn = false;
    d->stackOn = false;
    d->stackStream = nullptr;
}
void sfp_stack_stats(sfp_dev* d, uint64_t* merged, uint64_t* single) {
    if (merged) *merged = d->stkMerged;
    if (single) *single = d->stkSingle;
}
void sfp_lane_wait(sfp_dev* d, int waiter, int waitee) {
    if (waiter == waitee) return;
    const int keep = d->cur;
    d->cur = waitee;
    sfp_event* e = sfp_event_record(d);
    d->cur = waiter;
    sfp_event_wait(d, e);
    sfp_event_free(d, e);
    d->cur = keep;
}
const char* sfp_last_error(sfp_dev* d) {
    if (!d->capture) {  // (querying a capturing stream would invalidate the capture)
        hipError_t e = hipStreamQuery(d->st());
        if (e != hipSuccess && e != hipErrorNotReady) record(d, "stream", e);
    }
    std::lock_guard<std::mutex> g(d->mu);
    return d->err.empty() ? nullptr : d->err.c_str();
}

// ---- NTT ----
// FP64 butterflies for primes < 2^42 (SFHE_NTT_FP=0 runs every row on the
// integer path, which 60-bit primes always take)
static int nttFp() {
    static const int on = [] {
        const char* v = std::getenv("SFHE_NTT_FP");
        return (v ? std::atoi(v) : SFHE_NTT_FP) ? 1 : 0;
    }();
    return on;
}

// SFHE_NTT_SMALL_TILE (512 / 1024) and SFHE_NTT_SMALL_LE (2 / 3): the
// small-launch tile and register-round width (A/B knobs; defaults measured);
// SFHE_NTT_LE: register-round width experiments for big launches (2, 3, 4)
static uint32_t nttSmallTile() {
    static const uint32_t v = [] {
        const char* e = std::getenv("SFHE_NTT_SMALL_TILE");
        return e ? (uint32_t)std::atoi(e) : 1024u;
    }();
    return v;
}
static int nttSmallLe() {
    static const int v = [] {
        const char* e = std::getenv("SFHE_NTT_SMALL_LE");
        return e ? std::atoi(e) : 2;
    }();
    return v;
}
static int nttLe() {
    static const int v = [] {
        const char* e = std::getenv("SFHE_NTT_LE");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}

static RowGroup rowsOf(uint32_t P, uint32_t R, sfp_limbs pm) {
    RowGroup G;
    std::memset(&G, 0, sizeof G);
    G.P = P;
    G.R = R;
    G.pm = pm;
    return G;
}

// Would a forward NTT over `rows` rows take a two-stage (LE = 2) COL pass --
// the passes that have the inverse-COL prologue (RowGroup::icol)?  Mirrors
// nttRows' choice of path.  Off by default (SFHE_ICOL=1 turns it on).
static int nttLe();
static uint32_t nttSmallTile();
static int nttSmallLe();
static uint32_t nttT1kRows();
static bool icolPath(sfp_dev* d, uint32_t rows) {
    static const bool on = [] {  // (measured: sort 36.22 -> 36.63 ms with it on)
        const char* v = std::getenv("SFHE_ICOL");
        return v && *v == '1';
    }();
    if (!on || d->n <= (uint32_t)kNttTile) return false;
    const uint32_t st = nttSmallTile();
    const bool t1k = rows <= nttT1kRows() && d->n <= st * 128u;
    if (t1k) return nttSmallLe() == 2 && (st == 1024 || st == 512);
    const int le = nttLe();
    return (le ? le : (rows < (uint32_t)kNttSmallRows ? 2 : 3)) == 2;
}

// Both passes of a (batched) NTT over the rows of G -- or only the first
// (passes == 1: its output feeds a fused second pass, k_ntt_ks) or only the
// second (passes == 2: a fused kernel ran the first).
static uint32_t nttT1kRows() {
    static const uint32_t v = [] {
        const char* e = std::getenv("SFHE_NTT_T1K_ROWS");
        return e ? (uint32_t)std::atoi(e) : 64u;
    }();
    return v;
}
static int nttFp();
static void nttRows(sfp_dev* d, const RowGroup& G0, int inverse, int passes = 3) {
    const RowGroup& G = G0;
    const uint32_t rows = G.P * G.R;
    if (!rows || !limbsOk(d, G.pm, "ntt")) return;
    if (G.lift && G.liftPrime >= d->np) return (void)limbsOk(d, sfp_limbs{1, 1, G.liftPrime, G.liftPrime}, "ntt lift");
    const double bytes = 16.0 * rows * d->n;
    if (passes != 3 && d->n <= (uint32_t)kNttTile) {
        record(d, "ntt (a single pass: rings above one tile only)", hipErrorInvalidValue);
        return;
    }
    if (d->n <= (uint32_t)kNttTile) {  // small rings: one single-pass block per row
        timedLaunch(d, SFP_FAM_NTT, bytes, [&] {
            if (inverse)
                SFP_GO(k_ntt_small<true>, dim3(1, rows), dim3(kNttSmallThreads), G, d->bar,
                                   d->ipsi, d->ipsiS, d->ninv, d->ninvS, d->logn);
            else
                SFP_GO(k_ntt_small<false>, dim3(1, rows), dim3(kNttSmallThreads), G, d->bar,
                                   d->psi, d->psiS, d->ninv, d->ninvS, d->logn);
        });
        checkLaunch(d, "ntt");
        return;
    }
    const u64* tw = inverse ? d->ipsi : d->psi;
    const u64* twS = inverse ? d->ipsiS : d->psiS;
    const double* twD = inverse ? d->ipsiD : d->psiD;
    const double* rowD = inverse ? d->irowD : d->rowD;
    // Launches over few rows are latency-bound (a one-limb pass is one tile
    // round trip per block: ~1.5 us load, ~1 us per register round, tools/
    // microbench with SFHE_NTT_TRACE): up to SFHE_NTT_T1K_ROWS rows (default
    // 64) they run 1024-word tiles -- twice the blocks, half the work each;
    // needs >= 2 columns per COL tile, i.e. n <= 2^17.  Measured on the metric
    // sort: NTT 47.9 -> 46.0 ms, wall 58.1 -> 57.5 ms.
    const uint32_t t1kRows = nttT1kRows();
    const uint32_t smallTile = nttSmallTile();
    const int smallLe = nttSmallLe();
    const bool t1k = rows <= t1kRows && d->n <= smallTile * 128u;
    dim3 g(d->n / (t1k ? smallTile : (uint32_t)kNttTile), rows);
    uint32_t gridRows = rows;  // (k_modup_col: grid rows are groups of target rows)
    const bool small = rows < (uint32_t)kNttSmallRows;
    int npass = 0;
    // kern2 / kern4: the same pass over two / four row groups (merged launches), or null
    auto pass = [&](auto kern, NttKern2 kern2, NttKern4 kern4, NttKern8 kern8, int threads) {
        if (!((passes >> npass++) & 1)) return;
        timedLaunch(d, SFP_FAM_NTT, bytes, [&] {
            RowGroupSet<1> GS;
            GS.a[0] = G;
            GS.start[0] = 0;
            GS.inter = 0;
            const int fp = nttFp();
            StackRec r;
            r.go = [=](hipStream_t s_) {
                hipLaunchKernelGGL(kern, g, dim3(threads), 0, s_, GS, d->bar, tw, twS, d->ninv, d->ninvS, d->logn,
                                   twD, d->qinvD, d->ninvD, d->ninvQ, fp, rowD);
            };
            if (kern2 && d->stackOn) {
                auto P = std::make_shared<NttPay>();
                P->G = G;
                P->rows = gridRows;
                P->g = g;
                P->threads = threads;
                P->useFp = fp;
                P->k2 = kern2;
                P->k4 = kern4;
                P->k8 = kern8;
                P->tw = tw;
                P->twS = twS;
                P->twD = twD;
                P->rowD = rowD;
                r.cls = STK_NTT;
                r.key = stkKey((const void*)kern, g.x, (uint32_t)threads);
                r.pay = std::move(P);
            }
            issueRec(d, std::move(r));
        });
    };
    const int le = nttLe();
    const int L = le ? le : (small ? 2 : 3);
    constexpr int T = kNttTile;
    auto smallPasses = [&](auto tileC) {
        constexpr int ST = decltype(tileC)::value;
        if (smallLe == 3) {
            if (!inverse) {
                pass(k_ntt<false, true, 3, ST>, NttKern2{}, NttKern4{}, NttKern8{}, ST >> 3);
                pass(k_ntt<false, false, 3, ST>, NttKern2{}, NttKern4{}, NttKern8{}, ST >> 3);
            } else {
                pass(k_ntt<true, false, 3, ST>, NttKern2{}, NttKern4{}, NttKern8{}, ST >> 3);
                pass(k_ntt<true, true, 3, ST>, NttKern2{}, NttKern4{}, NttKern8{}, ST >> 3);
            }
        } else if (!inverse) {
            if (G.cy)  // ModUpPlan: the conversion in the COL pass's prologue (modupConvOk: LE 2, 1024-word tiles)
                pass(k_ntt<false, true, 2, ST, 1, true>, k_ntt<false, true, 2, ST, 2, true>,
                     k_ntt<false, true, 2, ST, 4, true>, k_ntt<false, true, 2, ST, 8, true>, ST >> 2);
            else if (G.icol)  // a rescale's lift with its source's inverse COL pass in the prologue
                pass(k_ntt<false, true, 2, ST, 1, false, true>, k_ntt<false, true, 2, ST, 2, false, true>,
                     k_ntt<false, true, 2, ST, 4, false, true>, k_ntt<false, true, 2, ST, 8, false, true>, ST >> 2);
            else
                pass(k_ntt<false, true, 2, ST>, k_ntt<false, true, 2, ST, 2>, k_ntt<false, true, 2, ST, 4>, k_ntt<false, true, 2, ST, 8>, ST >> 2);
            pass(k_ntt<false, false, 2, ST>, k_ntt<false, false, 2, ST, 2>, k_ntt<false, false, 2, ST, 4>, k_ntt<false, false, 2, ST, 8>, ST >> 2);
        } else {
            pass(k_ntt<true, false, 2, ST>, k_ntt<true, false, 2, ST, 2>, k_ntt<true, false, 2, ST, 4>, k_ntt<true, false, 2, ST, 8>, ST >> 2);
            pass(k_ntt<true, true, 2, ST>, k_ntt<true, true, 2, ST, 2>, k_ntt<true, true, 2, ST, 4>, k_ntt<true, true, 2, ST, 8>, ST >> 2);
        }
    };
    if (G.icol && (inverse || !icolPath(d, rows))) {
        record(d, "ntt: inverse-COL prologue outside its shape", hipErrorInvalidValue);
        return;
    }
    static const bool modupCol = [] {  // SFHE_MODUP_COL=0: k_ntt<..., CONV> (one target per block; A/B)
        const char* v = std::getenv("SFHE_MODUP_COL");
        return !v || *v != '0';
    }();
    if (G.md) {
        // ModDown (mdColArgs): its conversion + the COL pass, kModdownTg targets per block
        if (inverse || d->logn != 16 || smallTile != 1024 || L != 2 || passes != 3) {
            record(d, "ntt: fused ModDown pass outside its shape", hipErrorInvalidValue);
            return;
        }
        constexpr int TG = kModdownTg;
        g.y = G.P * ((G.R + TG - 1) / TG);
        gridRows = g.y;
        if (t1k)
            pass(k_moddown_col<1024, 1, TG>, k_moddown_col<1024, 2, TG>, k_moddown_col<1024, 4, TG>,
                 k_moddown_col<1024, 8, TG>, 1024 >> 2);
        else
            pass(k_moddown_col<T, 1, TG>, k_moddown_col<T, 2, TG>, k_moddown_col<T, 4, TG>, k_moddown_col<T, 8, TG>,
                 T >> 2);
        g.y = rows;
        gridRows = rows;
        if (t1k)
            pass(k_ntt<false, false, 2, 1024>, k_ntt<false, false, 2, 1024, 2>, k_ntt<false, false, 2, 1024, 4>,
                 k_ntt<false, false, 2, 1024, 8>, 1024 >> 2);
        else
            pass(k_ntt<false, false, 2, T>, k_ntt<false, false, 2, T, 2>, k_ntt<false, false, 2, T, 4>,
                 k_ntt<false, false, 2, T, 8>, T >> 2);
    } else if (G.cy && modupCol && !inverse && d->logn == 16 && smallTile == 1024 && L == 2) {
        // ModUpPlan at ring 2^16: the conversion + COL pass, kModupTg targets per block
        // small launches (fewer than SFHE_MODUP_TG_SMALL blocks at kModupTg
        // targets per block, default 512: two per CU) take two targets per
        // block -- twice the blocks, half of each block's serial target chain
        constexpr int TG = kModupTg;
        static const uint32_t tgSmall = [] {
            const char* v = std::getenv("SFHE_MODUP_TG_SMALL");
            return v ? (uint32_t)std::atoi(v) : 512u;
        }();
        const bool tg2 = G.P * ((G.R + TG - 1) / TG) * g.x < tgSmall;
        const int tg = tg2 ? 2 : TG;
        g.y = G.P * ((G.R + tg - 1) / tg);
        gridRows = g.y;
        // (each specialisation named in a call of its own: named only inside a
        // conditional expression, the device code of some was never emitted --
        // "Cannot find Symbol" at launch)
        if (t1k && tg2)
            pass(k_modup_col<1024, 1, 2>, k_modup_col<1024, 2, 2>, k_modup_col<1024, 4, 2>, k_modup_col<1024, 8, 2>,
                 1024 >> 2);
        else if (t1k)
            pass(k_modup_col<1024, 1, TG>, k_modup_col<1024, 2, TG>, k_modup_col<1024, 4, TG>, k_modup_col<1024, 8, TG>,
                 1024 >> 2);
        else if (tg2)
            pass(k_modup_col<T, 1, 2>, k_modup_col<T, 2, 2>, k_modup_col<T, 4, 2>, k_modup_col<T, 8, 2>, T >> 2);
        else
            pass(k_modup_col<T, 1, TG>, k_modup_col<T, 2, TG>, k_modup_col<T, 4, TG>, k_modup_col<T, 8, TG>, T >> 2);
        g.y = rows;
        gridRows = rows;
        if (t1k)
            pass(k_ntt<false, false, 2, 1024>, k_ntt<false, false, 2, 1024, 2>, k_ntt<false, false, 2, 1024, 4>,
                 k_ntt<false, false, 2, 1024, 8>, 1024 >> 2);
        else
            pass(k_ntt<false, false, 2, T>, k_ntt<false, false, 2, T, 2>, k_ntt<false, false, 2, T, 4>,
                 k_ntt<false, false, 2, T, 8>, T >> 2);
    } else if (t1k) {
        if (smallTile == 512)
            smallPasses(std::integral_constant<int, 512>{});
        else
            smallPasses(std::integral_constant<int, 1024>{});
    } else if (!inverse) {
        if (L == 4) {
            pass(k_ntt<false, true, 4, T>, NttKern2{}, NttKern4{}, NttKern8{}, T >> 4);
            pass(k_ntt<false, false, 4, T>, NttKern2{}, NttKern4{}, NttKern8{}, T >> 4);
        } else if (L == 2) {
            if (G.cy)
                pass(k_ntt<false, true, 2, T, 1, true>, k_ntt<false, true, 2, T, 2, true>,
                     k_ntt<false, true, 2, T, 4, true>, k_ntt<false, true, 2, T, 8, true>, T >> 2);
            else if (G.icol)
                pass(k_ntt<false, true, 2, T, 1, false, true>, k_ntt<false, true, 2, T, 2, false, true>,
                     k_ntt<false, true, 2, T, 4, false, true>, k_ntt<false, true, 2, T, 8, false, true>, T >> 2);
            else
                pass(k_ntt<false, true, 2, T>, k_ntt<false, true, 2, T, 2>, k_ntt<false, true, 2, T, 4>, k_ntt<false, true, 2, T, 8>, T >> 2);
            pass(k_ntt<false, false, 2, T>, k_ntt<false, false, 2, T, 2>, k_ntt<false, false, 2, T, 4>, k_ntt<false, false, 2, T, 8>, T >> 2);
        } else {
            pass(k_ntt<false, true, 3, T>, NttKern2{}, NttKern4{}, NttKern8{}, T >> 3);
            pass(k_ntt<false, false, 3, T>, NttKern2{}, NttKern4{}, NttKern8{}, T >> 3);
        }
    } else {
        if (L == 4) {
            pass(k_ntt<true, false, 4, T>, NttKern2{}, NttKern4{}, NttKern8{}, T >> 4);
            pass(k_ntt<true, true, 4, T>, NttKern2{}, NttKern4{}, NttKern8{}, T >> 4);
        } else if (L == 2) {
            pass(k_ntt<true, false, 2, T>, k_ntt<true, false, 2, T, 2>, k_ntt<true, false, 2, T, 4>, k_ntt<true, false, 2, T, 8>, T >> 2);
            pass(k_ntt<true, true, 2, T>, k_ntt<true, true, 2, T, 2>, k_ntt<true, true, 2, T, 4>, k_ntt<true, true, 2, T, 8>, T >> 2);
        } else {
            pass(k_ntt<true, false, 3, T>, NttKern2{}, NttKern4{}, NttKern8{}, T >> 3);
            pass(k_ntt<true, true, 3, T>, NttKern2{}, NttKern4{}, NttKern8{}, T >> 3);
        }
    }
    checkLaunch(d, "ntt");
}

void sfp_ntt(sfp_dev* d, uint64_t* p, sfp_limbs m, int inverse) {
    RowGroup G = rowsOf(1, m.count, m);
    G.src = G.dst = RowPtr{p, 0, (long long)d->n};
    nttRows(d, G, inverse);
}

void sfp_ntt_batch(sfp_dev* d, uint64_t* p, size_t stride, uint32_t count, sfp_limbs m, int inverse) {
    if (!count) return;
    RowGroup G = rowsOf(count, m.count, m);
    G.src = G.dst = RowPtr{p, (long long)stride, (long long)d->n};
    nttRows(d, G, inverse);
}

// Developer hook (SFHE_NTT_TRACE builds): k_mdrsf's FP64 blocks' phase clocks
// since the last call -- [0] loads + constants, [1] phase 1 (y), [2] the
// overflow and the dropped row, [3] phase 2 and the stores, [7] blocks; -1
// otherwise.
extern "C" int sfp_mdrs_trace(sfp_dev* d, unsigned long long* out8) {
#ifdef SFHE_NTT_TRACE
    syncAll(d);
    static unsigned long long all[kTraceSlots * 8];
    SFP_CHECK(hipMemcpyFromSymbol(all, HIP_SYMBOL(g_mdrsTrace), sizeof all));
    for (int i = 0; i < 8; ++i) {
        out8[i] = 0;
        for (int k = 0; k < kTraceSlots; ++k) out8[i] += all[k * 8 + i];
    }
    static const unsigned long long zero[kTraceSlots * 8] = {};
    SFP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_mdrsTrace), zero, sizeof zero));
    return 0;
#else
    (void)d;
    (void)out8;
    return -1;
#endif
}

// Developer hook (SFHE_NTT_TRACE builds): per-kernel phase clocks since the
// last call, [variant INV*2+COL][phase 0..5, 7 = blocks]; -1 otherwise.
extern "C" int sfp_ntt_trace(sfp_dev* d, unsigned long long* out32) {
#ifdef SFHE_NTT_TRACE
    syncAll(d);
    static unsigned long long all[kTraceSlots * 32];
    SFP_CHECK(hipMemcpyFromSymbol(all, HIP_SYMBOL(g_nttTrace), sizeof all));
    for (int i = 0; i < 32; ++i) {
        out32[i] = 0;
        for (int k = 0; k < kTraceSlots; ++k) out32[i] += all[k * 32 + i];
    }
    static const unsigned long long zero[kTraceSlots * 32] = {};
    SFP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_nttTrace), zero, sizeof zero));
    return 0;
#else
    (void)d;
    (void)out32;
    return -1;
#endif
}

void sfp_prof_set(sfp_dev* d, uint32_t fam, uint32_t period) {
    if (fam >= SFP_FAM_COUNT) return;
    auto& f = d->prof[fam];
    profFlush(d, f);
    f = sfp_dev::ProfFam{};
    f.period = period;
}

// ---- graph capture ----
int sfp_capture_begin(sfp_dev* d) {
    if (d->capture) {
        record(d, "capture_begin (a capture is already open)", hipErrorInvalidValue);
        return -1;
    }
    syncAll(d);
    d->cur = 0;
    auto* g = new sfp_graph;
    const hipError_t e = hipStreamBeginCapture(d->streams[0], hipStreamCaptureModeRelaxed);
    if (e != hipSuccess) {
        hipGetLastError();
        delete g;
        std::fprintf(stderr, "sfhe: hipStreamBeginCapture: %s\n", hipGetErrorString(e));
        return -1;
    }
    d->capture = g;
    return 0;
}

int sfp_capturing(sfp_dev* d) { return d->capture != nullptr; }

void sfp_graph_destroy(sfp_dev* d, sfp_graph* g) {
    if (!g) return;
    if (!d->capture) syncAll(d);
    if (g->exec) hipGraphExecDestroy(g->exec);
    if (g->g) hipGraphDestroy(g->g);
    for (auto& c : g->arena) hipFree(c.dev);
    delete g;
}

void sfp_clear_error(sfp_dev* d) {
    std::lock_guard<std::mutex> g(d->mu);
    d->err.clear();
}

sfp_graph* sfp_capture_end(sfp_dev* d) {
    sfp_graph* g = d->capture;
    if (!g) return nullptr;
    stackFlush(d);  // (a stacked region left open: its launches belong to the graph)
    d->cur = 0;
    // test knob (read per capture): abandon this capture as if it had failed
    if (const char* f = std::getenv("SFHE_CAPTURE_FORCE_FAIL"); f && *f == '1') captureFail(d, "forced (SFHE_CAPTURE_FORCE_FAIL)");
    const hipError_t e = hipStreamEndCapture(d->streams[0], &g->g);
    d->capture = nullptr;
    if (e != hipSuccess || g->failed || !g->g) {
        hipGetLastError();
        std::string why = g->failed ? g->why : std::string("hipStreamEndCapture: ") + hipGetErrorString(e);
        sfp_graph_destroy(d, g);
        std::lock_guard<std::mutex> lk(d->mu);
        if (d->err.empty()) d->err = "graph capture failed: " + why;
        return nullptr;
    }
    for (auto& c : g->arena) hostToDev(d, c.dev, c.host.data(), c.used * 8);
    if (hipGraphGetNodes(g->g, nullptr, &g->nodes) != hipSuccess) g->nodes = 0;
    static const size_t maxNodes = [] {  // SFHE_GRAPH_MAX_NODES: larger captures fall back to eager
        const char* v = std::getenv("SFHE_GRAPH_MAX_NODES");
        return v ? (size_t)std::atoll(v) : (size_t)600000;  // (the k-way sort: ~225 k)
    }();
    if (std::getenv("SFHE_GRAPH_DEBUG")) std::fprintf(stderr, "[sfhe] captured graph: %zu nodes\n", g->nodes);
    if (g->nodes > maxNodes) {
        sfp_graph_destroy(d, g);
        std::lock_guard<std::mutex> lk(d->mu);
        if (d->err.empty()) d->err = "graph capture failed: more nodes than SFHE_GRAPH_MAX_NODES";
        return nullptr;
    }
    if (hipGraphInstantiate(&g->exec, g->g, nullptr, nullptr, 0) != hipSuccess) {
        const hipError_t ie = hipGetLastError();
        sfp_graph_destroy(d, g);
        record(d, "hipGraphInstantiate", ie);
        return nullptr;
    }
    return g;
}

void sfp_graph_launch(sfp_dev* d, sfp_graph* g) {
    if (!g || !g->exec) return record(d, "graph_launch", hipErrorInvalidValue);
    hipGraphExec_t ex = g->exec;
    issue(d, [d, ex](hipStream_t s_) { SFP_CHECK(hipGraphLaunch(ex, s_)); });
}

size_t sfp_graph_nodes(const sfp_graph* g) { return g ? g->nodes : 0; }

// The family of a kernel (graph timing): every instantiation the launch
// sites issue; anything else is SFP_FAM_COUNT ("other").
template <bool I, bool C, int LE, int T>
static void addNtt(std::unordered_map<const void*, uint32_t>& m, bool merged) {
    m[(const void*)k_ntt<I, C, LE, T>] = SFP_FAM_NTT;
    if (merged) {
        m[(const void*)k_ntt<I, C, LE, T, 2>] = SFP_FAM_NTT;
        m[(const void*)k_ntt<I, C, LE, T, 4>] = SFP_FAM_NTT;
        m[(const void*)k_ntt<I, C, LE, T, 8>] = SFP_FAM_NTT;
    }
}
template <int LE, int T>
static void addNttAll(std::unordered_map<const void*, uint32_t>& m, bool merged) {
    addNtt<false, true, LE, T>(m, merged);
    addNtt<false, false, LE, T>(m, merged);
    addNtt<true, true, LE, T>(m, merged);
    addNtt<true, false, LE, T>(m, merged);
}
static uint32_t kernelFamily(const void* f) {
    static const std::unordered_map<const void*, uint32_t> fam = [] {
        std::unordered_map<const void*, uint32_t> m;
        addNttAll<2, kNttTile>(m, true);
        for (const void* k : {(const void*)k_ntt<false, true, 2, kNttTile, 1, true>,
                              (const void*)k_ntt<false, true, 2, kNttTile, 2, true>,
                              (const void*)k_ntt<false, true, 2, kNttTile, 4, true>,
                              (const void*)k_ntt<false, true, 2, kNttTile, 8, true>,
                              (const void*)k_ntt<false, true, 2, 1024, 1, true>, (const void*)k_ntt<false, true, 2, 1024, 2, true>,
                              (const void*)k_ntt<false, true, 2, 1024, 4, true>, (const void*)k_ntt<false, true, 2, 1024, 8, true>})
            m[k] = SFP_FAM_NTT;  // (the ModUp COL pass with its conversion)
        for (const void* k : {(const void*)k_ntt<false, true, 2, kNttTile, 1, false, true>,
                              (const void*)k_ntt<false, true, 2, kNttTile, 2, false, true>,
                              (const void*)k_ntt<false, true, 2, kNttTile, 4, false, true>,
                              (const void*)k_ntt<false, true, 2, kNttTile, 8, false, true>,
                              (const void*)k_ntt<false, true, 2, 1024, 1, false, true>,
                              (const void*)k_ntt<false, true, 2, 1024, 2, false, true>,
                              (const void*)k_ntt<false, true, 2, 1024, 4, false, true>,
                              (const void*)k_ntt<false, true, 2, 1024, 8, false, true>,
                              (const void*)k_ntt<false, true, 2, 512, 1, false, true>,
                              (const void*)k_ntt<false, true, 2, 512, 2, false, true>,
                              (const void*)k_ntt<false, true, 2, 512, 4, false, true>,
                              (const void*)k_ntt<false, true, 2, 512, 8, false, true>})
            m[k] = SFP_FAM_NTT;  // (a rescale's lift pass with its source's inverse COL pass: a row's read + write)
        for (const void* k : {(const void*)k_modup_col<kNttTile, 1, kModupTg>, (const void*)k_modup_col<kNttTile, 2, kModupTg>,
                              (const void*)k_modup_col<kNttTile, 4, kModupTg>, (const void*)k_modup_col<kNttTile, 8, kModupTg>,
                              (const void*)k_modup_col<1024, 1, kModupTg>, (const void*)k_modup_col<1024, 2, kModupTg>,
                              (const void*)k_modup_col<1024, 4, kModupTg>, (const void*)k_modup_col<1024, 8, kModupTg>,
                              (const void*)k_modup_col<kNttTile, 1, 2>, (const void*)k_modup_col<kNttTile, 2, 2>,
                              (const void*)k_modup_col<kNttTile, 4, 2>, (const void*)k_modup_col<kNttTile, 8, 2>,
                              (const void*)k_modup_col<1024, 1, 2>, (const void*)k_modup_col<1024, 2, 2>,
                              (const void*)k_modup_col<1024, 4, 2>, (const void*)k_modup_col<1024, 8, 2>})
            m[k] = SFP_FAM_NTT;
        for (const void* k : {(const void*)k_moddown_col<kNttTile, 1, kModdownTg>, (const void*)k_moddown_col<kNttTile, 2, kModdownTg>,
                              (const void*)k_moddown_col<kNttTile, 4, kModdownTg>, (const void*)k_moddown_col<kNttTile, 8, kModdownTg>,
                              (const void*)k_moddown_col<1024, 1, kModdownTg>, (const void*)k_moddown_col<1024, 2, kModdownTg>,
                              (const void*)k_moddown_col<1024, 4, kModdownTg>, (const void*)k_moddown_col<1024, 8, kModdownTg>})
            m[k] = SFP_FAM_NTT;
        addNttAll<2, 1024>(m, true);
        addNttAll<2, 512>(m, true);
        addNttAll<3, kNttTile>(m, false);
        addNttAll<4, kNttTile>(m, false);
        addNttAll<3, 1024>(m, false);
        addNttAll<3, 512>(m, false);
        for (const void* k : {(const void*)k_convf<13>, (const void*)k_convf<16>, (const void*)k_convf<kMaxConvSrc>,
                              (const void*)k_conv, (const void*)k_mdrsf<13, true>, (const void*)k_mdrsf<16, true>,
                              (const void*)k_mdrsf<kMaxConvSrc, true>, (const void*)k_mdrsf<13>,
                              (const void*)k_mdrsf<16>, (const void*)k_mdrsf<kMaxConvSrc>, (const void*)k_conv_mdrs,
                              (const void*)k_mdrsi<16>, (const void*)k_mdrsi<kMaxConvSrc>})
            m[k] = SFP_FAM_CONV;
        for (const void* k : {(const void*)k_ks_inner<1>, (const void*)k_ks_inner<2>, (const void*)k_ks_inner<4>})
            m[k] = SFP_FAM_KSINNER;
        for (const void* k : {(const void*)k_ntt_ks<2, 1024>, (const void*)k_ntt_ks<2, 1024, 2>,
                              (const void*)k_ntt_ks<2, 1024, 4>, (const void*)k_ntt_ks<2, 1024, 8>,
                              (const void*)k_ntt_ks<2, kNttTile>, (const void*)k_ntt_ks<2, kNttTile, 2>,
                              (const void*)k_ntt_ks<2, kNttTile, 4>, (const void*)k_ntt_ks<2, kNttTile, 8>})
            m[k] = SFP_FAM_NTTKS;
        return m;
    }();
    auto it = fam.find(f);
    return it == fam.end() ? (uint32_t)SFP_FAM_COUNT : it->second;
}

// An NTT-family node's algorithmic bytes in rows of 16n bytes (one row read
// and written): its grid rows, except for the fused conversion passes, read
// from their argument sets, which read their sources once and write their
// targets once -- k_modup_col: per digit its own rows in, the other R - own
// rows out (R / 2 rows of 16n); k_moddown_col: per polynomial the cRows
// source rows (K P rows, + the dropped row with the rescale) in, R rows out.
template <int NG>
static double fusedColRows(const void* arg, bool moddown) {
    const auto& S = *static_cast<const RowGroupSet<NG>*>(arg);
    double r = 0;
    for (int i = 0; i < NG; ++i) {
        const RowGroup& G = S.a[i];
        r += moddown ? 0.5 * G.P * (G.R + G.cRows) : 0.5 * G.P * G.R;
    }
    return r;
}
template <int NG>
static bool isFusedCol(const void* f, bool md) {
    return md ? (f == (const void*)k_moddown_col<kNttTile, NG, kModdownTg> ||
                 f == (const void*)k_moddown_col<1024, NG, kModdownTg>)
              : (f == (const void*)k_modup_col<kNttTile, NG, kModupTg> || f == (const void*)k_modup_col<1024, NG, kModupTg> ||
                 f == (const void*)k_modup_col<kNttTile, NG, 2> || f == (const void*)k_modup_col<1024, NG, 2>);
}
static double nttNodeRows(const hipKernelNodeParams& kp) {
    const void* f = kp.func;
    if (kp.kernelParams) {
        for (bool md : {false, true}) {
            if (isFusedCol<1>(f, md)) return fusedColRows<1>(kp.kernelParams[0], md);
            if (isFusedCol<2>(f, md)) return fusedColRows<2>(kp.kernelParams[0], md);
            if (isFusedCol<4>(f, md)) return fusedColRows<4>(kp.kernelParams[0], md);
            if (isFusedCol<8>(f, md)) return fusedColRows<8>(kp.kernelParams[0], md);
        }
    }
    return (double)kp.gridDim.y;
}

// A conversion-family node's algorithmic bytes (8n per source row read and
// per target row written): k_mdrsf / k_conv_mdrs per polynomial (grid row)
// the K source rows and the dropped row in, l target rows out; k_convf /
// k_conv per job its ns sources in, its ntUse targets out.
static double convNodeBytes(const hipKernelNodeParams& kp, uint32_t n) {
    const void* f = kp.func;
    if (!kp.kernelParams) return 0;
    const bool mdrs = f == (const void*)k_mdrsf<13> || f == (const void*)k_mdrsf<16> ||
                      f == (const void*)k_mdrsf<kMaxConvSrc> || f == (const void*)k_mdrsf<13, true> ||
                      f == (const void*)k_mdrsf<16, true> || f == (const void*)k_mdrsf<kMaxConvSrc, true> ||
                      f == (const void*)k_conv_mdrs || f == (const void*)k_mdrsi<16> ||
                      f == (const void*)k_mdrsi<kMaxConvSrc>;
    if (mdrs) {
        const MdrsArgs& A = *static_cast<const MdrsArgs*>(kp.kernelParams[0]);
        return 8.0 * n * kp.gridDim.y * (A.ns + 1.0 + A.l);
    }
    const ConvJobs& J = *static_cast<const ConvJobs*>(kp.kernelParams[0]);
    double r = 0;
    for (uint32_t j = 0; j < kp.gridDim.y && j < (uint32_t)kMaxConvJobs; ++j) r += J.j[j].ns + (double)J.j[j].ntUse;
    return 8.0 * n * r;
}
// k_ntt_ks: per extended row, beta ext rows + 2 beta key rows in, two
// accumulator rows out (+ two in when accumulating)
template <int NG>
static double ksNodeBytesNG(const void* arg, uint32_t gridY, uint32_t n) {
    const auto& S = *static_cast<const ArgSet<KsArgs, NG>*>(arg);
    double b = 0;
    for (int i = 0; i < NG; ++i) {
        const uint32_t r0 = S.start[i], r1 = i + 1 < NG ? S.start[i + 1] : gridY;
        const uint32_t rows = S.inter ? gridY / NG : (r1 > r0 ? r1 - r0 : 0);  // (unused sets: none)
        b += 8.0 * n * rows * (3.0 * S.a[i].beta + (S.a[i].accum ? 4.0 : 2.0));
    }
    return b;
}
static double ksNodeBytes(const hipKernelNodeParams& kp, uint32_t n) {
    const void* f = kp.func;
    if (!kp.kernelParams) return 0;
    if (f == (const void*)k_ntt_ks<2, 1024> || f == (const void*)k_ntt_ks<2, kNttTile>)
        return ksNodeBytesNG<1>(kp.kernelParams[0], kp.gridDim.y, n);
    if (f == (const void*)k_ntt_ks<2, 1024, 2> || f == (const void*)k_ntt_ks<2, kNttTile, 2>)
        return ksNodeBytesNG<2>(kp.kernelParams[0], kp.gridDim.y, n);
    if (f == (const void*)k_ntt_ks<2, 1024, 4> || f == (const void*)k_ntt_ks<2, kNttTile, 4>)
        return ksNodeBytesNG<4>(kp.kernelParams[0], kp.gridDim.y, n);
    return ksNodeBytesNG<8>(kp.kernelParams[0], kp.gridDim.y, n);
}

int sfp_graph_family_time(sfp_dev* d, sfp_graph* g, uint32_t fam, int reps, double* ms, uint64_t* launches,
                          double* bytes) {
    if (!g || !g->g || fam > SFP_FAM_ALL || reps < 1 || d->capture) return -1;
    size_t nn = 0;
    if (hipGraphGetNodes(g->g, nullptr, &nn) != hipSuccess) return -1;
    std::vector<hipGraphNode_t> nodes(nn);
    if (hipGraphGetNodes(g->g, nodes.data(), &nn) != hipSuccess) return -1;
    // capture order = topological order of a stream capture; keep it
    hipGraph_t sub = nullptr;
    if (hipGraphCreate(&sub, 0) != hipSuccess) return -1;
    hipGraphNode_t prev = nullptr;
    uint64_t cnt = 0;
    double b = 0;
    for (hipGraphNode_t nd : nodes) {
        hipGraphNodeType t;
        if (hipGraphNodeGetType(nd, &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
        hipKernelNodeParams kp;
        std::memset(&kp, 0, sizeof kp);
        if (hipGraphKernelNodeGetParams(nd, &kp) != hipSuccess) continue;
        if (!kp.func || (!kp.kernelParams && !kp.extra)) {  // (a tool may rewrite the nodes)
            hipGraphDestroy(sub);
            return -1;
        }
        const uint32_t kf = kernelFamily(kp.func);
        if (fam != SFP_FAM_ALL && kf != fam) continue;
        hipGraphNode_t nn2 = nullptr;
        if (hipGraphAddKernelNode(&nn2, sub, prev ? &prev : nullptr, prev ? 1 : 0, &kp) != hipSuccess) {
            hipGraphDestroy(sub);
            return -1;
        }
        prev = nn2;
        ++cnt;
        if (kf == SFP_FAM_NTT) b += 16.0 * nttNodeRows(kp) * d->n;  // one pass reads and writes each row once
        if (kf == SFP_FAM_CONV && fam == SFP_FAM_CONV) b += convNodeBytes(kp, d->n);
        if (kf == SFP_FAM_NTTKS && fam == SFP_FAM_NTTKS) b += ksNodeBytes(kp, d->n);
    }
    hipGraphExec_t ex = nullptr;
    if (!cnt || hipGraphInstantiate(&ex, sub, nullptr, nullptr, 0) != hipSuccess) {
        hipGetLastError();
        hipGraphDestroy(sub);
        return -1;
    }
    syncAll(d);
    hipEvent_t e0 = takeEvent(d), e1 = takeEvent(d);
    SFP_CHECK(hipGraphLaunch(ex, d->st()));  // warm
    SFP_CHECK(hipEventRecord(e0, d->st()));
    for (int r = 0; r < reps; ++r) SFP_CHECK(hipGraphLaunch(ex, d->st()));
    SFP_CHECK(hipEventRecord(e1, d->st()));
    SFP_CHECK(hipEventSynchronize(e1));
    float t = 0;
    SFP_CHECK(hipEventElapsedTime(&t, e0, e1));
    d->evPool.push_back(e0);
    d->evPool.push_back(e1);
    hipGraphExecDestroy(ex);
    hipGraphDestroy(sub);
    if (ms) *ms = t / reps;
    if (launches) *launches = cnt;
    if (bytes) *bytes = b;
    return 0;
}

void sfp_serialize(sfp_dev* d, int on) {
    syncAll(d);
    d->serial = on != 0;
}

int sfp_prof_read(sfp_dev* d, uint32_t fam, uint64_t* launches, uint64_t* timed, double* ms,
                  double* bytes) {
    if (fam >= SFP_FAM_COUNT) return -1;
    auto& f = d->prof[fam];
    profFlush(d, f);
    if (launches) *launches = f.seen;
    if (timed) *timed = f.timed;
    if (ms) *ms = f.ms;
    if (bytes) *bytes = f.bytes;
    return 0;
}

// ---- elementwise ----
template <int OP>
static void ew(sfp_dev* d, u64* out, const u64* a, const u64* b, const u64* c, sfp_limbs m,
               const u64* k) {
    if (!m.count || !limbsOk(d, m, "elementwise")) return;
    ConstArgs ka;
    if (k) std::memcpy(ka.k, k, m.count * 8);
    const size_t pairs = ((size_t)m.count * d->n) / 2;
    EwArgs A{out, a, b, c, m, {}};
    A.k = ka;
    issueY<EwArgs>(d, k_ew<OP, 1>, k_ew<OP, 2>, k_ew<OP, 4>, dim3(ewGrid(pairs)), A);
    checkLaunch(d, "elementwise");
}

void sfp_add(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m) {
    ew<EW_ADD>(d, out, a, b, nullptr, m, nullptr);
}
void sfp_sub(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m) {
    ew<EW_SUB>(d, out, a, b, nullptr, m, nullptr);
}
void sfp_neg(sfp_dev* d, uint64_t* out, const uint64_t* a, sfp_limbs m) {
    ew<EW_NEG>(d, out, a, nullptr, nullptr, m, nullptr);
}
void sfp_mul(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b, sfp_limbs m) {
    ew<EW_MUL>(d, out, a, b, nullptr, m, nullptr);
}
void sfp_mul_add(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* b,
                 const uint64_t* c, sfp_limbs m) {
    ew<EW_MULADD>(d, out, a, b, c, m, nullptr);
}
void sfp_mul_const(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* k, sfp_limbs m) {
    ew<EW_MULC>(d, out, a, nullptr, nullptr, m, k);
}
void sfp_add_const(sfp_dev* d, uint64_t* out, const uint64_t* a, const uint64_t* k, sfp_limbs m) {
    ew<EW_ADDC>(d, out, a, nullptr, nullptr, m, k);
}

void sfp_tensor(sfp_dev* d, uint64_t* d0, uint64_t* d1, uint64_t* d2, const uint64_t* a0,
                const uint64_t* a1, const uint64_t* b0, const uint64_t* b1, sfp_limbs m) {
    if (!limbsOk(d, m, "tensor")) return;
    const size_t total = (size_t)m.count * d->n;
    SFP_GO(k_tensor, dim3(ewGrid(total / 2)), dim3(kThreads), d0, d1, d2, a0, a1,
                       b0, b1, m, d->bar, d->logn);
    checkLaunch(d, "tensor");
}

void sfp_lin_wsum(sfp_dev* d, uint64_t* out, const uint64_t* const* ins, const uint64_t* k,
                  uint32_t nin, sfp_limbs m) {
    if (!limbsOk(d, m, "lin_wsum")) return;
    if (nin > SFP_MAX_WSUM) {
        record(d, "lin_wsum", hipErrorInvalidValue);
        return;
    }
    PtrList pl;
    for (uint32_t j = 0; j < nin; ++j) pl.p[j] = ins[j];
    const u64* dk = (const u64*)ringPut(d, k, (size_t)nin * m.count * 8);
    const size_t total = (size_t)m.count * d->n;
    issueY<WsumArgs>(d, k_lin_wsum<1>, k_lin_wsum<2>, k_lin_wsum<4>, dim3(ewGrid(total)), WsumArgs{out, pl, dk, nin, m});
    checkLaunch(d, "lin_wsum");
}

void sfp_lin_wsum_multi(sfp_dev* d, uint64_t* out, size_t outStride, size_t polyStride,
                        const uint64_t* const* in0, const uint64_t* const* in1, uint32_t nin,
                        const uint64_t* k, uint32_t nout, sfp_limbs m) {
    if (!nout || !nin || !m.count) return;
    if (nin > SFP_MAX_WSUM || !limbsOk(d, m, "lin_wsum_multi")) {
        record(d, "lin_wsum_multi", hipErrorInvalidValue);
        return;
    }
    PtrList2 pl;
    for (uint32_t j = 0; j < nin; ++j) {
        pl.a[j] = in0[j];
        pl.b[j] = in1[j];
    }
    const u64* dk = (const u64*)ringPut(d, k, (size_t)nout * nin * m.count * 8);
    const dim3 g((d->n / kThreads) * ((nout + kWsumChunk - 1) / kWsumChunk), m.count);
    SFP_GO(k_lin_wsum_multi, g, dim3(kThreads), out, outStride, polyStride, pl, dk,
                       nin, nout, m, d->bar, d->logn, d->qinvD, (int)nttFp());
    checkLaunch(d, "lin_wsum_multi");
}

void sfp_mac_plain2(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* const* a0,
                    const uint64_t* const* a1, const uint64_t* const* b, uint32_t nin, sfp_limbs m) {
    if (!m.count || !nin) return;
    if (!limbsOk(d, m, "mac_plain2")) return;
    if (nin > SFP_MAX_WSUM) {
        record(d, "mac_plain2", hipErrorInvalidValue);
        return;
    }
    PtrList3 L;
    for (uint32_t j = 0; j < nin; ++j) {
        L.a[j] = a0[j];
        L.c[j] = a1[j];
        L.b[j] = b[j];
    }
    const size_t total = (size_t)m.count * d->n;
    SFP_GO(k_mac_plain2, dim3(ewGrid(total / 2)), dim3(kThreads), out0, out1, L, nin, m,
                       d->bar, d->logn, d->qinvD);
    checkLaunch(d, "mac_plain2");
}

int sfp_mac_plain2_multi(sfp_dev* d, uint64_t* const* out0, uint64_t* const* out1, const uint64_t* const* a0,
                         const uint64_t* const* a1, const uint64_t* const* b, uint32_t nin, uint32_t ng,
                         sfp_limbs m) {
    if (!ng || ng > SFP_MAC_MULTI_G || !nin || nin > SFP_MAC_MULTI_N) return -1;
    if (!m.count) return 0;
    if (!limbsOk(d, m, "mac_plain2_multi")) return 0;
    PtrListM L;
    std::memset(&L, 0, sizeof L);
    for (uint32_t j = 0; j < nin; ++j) {
        L.a[j] = a0[j];
        L.c[j] = a1[j];
        for (uint32_t g = 0; g < ng; ++g) L.b[g * nin + j] = b[(size_t)g * nin + j];
    }
    for (uint32_t g = 0; g < ng; ++g) {
        L.o0[g] = out0[g];
        L.o1[g] = out1[g];
    }
    const size_t total = (size_t)m.count * d->n;
    const dim3 grid(ewGrid(total / 2));
    // (each specialisation launched by name: see tests/test_kernel_symbols.py)
    switch (ng) {
        case 1: SFP_GO(k_mac_plain2_multi<1>, grid, dim3(kThreads), L, nin, m, d->bar, d->logn, d->qinvD); break;
        case 2: SFP_GO(k_mac_plain2_multi<2>, grid, dim3(kThreads), L, nin, m, d->bar, d->logn, d->qinvD); break;
        case 3: SFP_GO(k_mac_plain2_multi<3>, grid, dim3(kThreads), L, nin, m, d->bar, d->logn, d->qinvD); break;
        case 4: SFP_GO(k_mac_plain2_multi<4>, grid, dim3(kThreads), L, nin, m, d->bar, d->logn, d->qinvD); break;
        case 5: SFP_GO(k_mac_plain2_multi<5>, grid, dim3(kThreads), L, nin, m, d->bar, d->logn, d->qinvD); break;
        case 6: SFP_GO(k_mac_plain2_multi<6>, grid, dim3(kThreads), L, nin, m, d->bar, d->logn, d->qinvD); break;
        case 7: SFP_GO(k_mac_plain2_multi<7>, grid, dim3(kThreads), L, nin, m, d->bar, d->logn, d->qinvD); break;
        default: SFP_GO(k_mac_plain2_multi<8>, grid, dim3(kThreads), L, nin, m, d->bar, d->logn, d->qinvD); break;
    }
    checkLaunch(d, "mac_plain2_multi");
    return 0;
}

void sfp_mac_plain(sfp_dev* d, uint64_t* out, const uint64_t* const* a, const uint64_t* const* b,
                   uint32_t nin, sfp_limbs m) {
    if (!limbsOk(d, m, "mac_plain")) return;
    if (nin > SFP_MAX_WSUM) {
        record(d, "mac_plain", hipErrorInvalidValue);
        return;
    }
    PtrList2 pl;
    for (uint32_t j = 0; j < nin; ++j) {
        pl.a[j] = a[j];
        pl.b[j] = b[j];
    }
    const size_t total = (size_t)m.count * d->n;
    SFP_GO(k_mac_plain, dim3(ewGrid(total)), dim3(kThreads), out, pl, nin, m,
                       d->bar, d->logn);
    checkLaunch(d, "mac_plain");
}

void sfp_automorph(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t g, sfp_limbs m) {
    const size_t total = (size_t)m.count * d->n;
    issueY<AutArgs>(d, k_automorph<1>, k_automorph<2>, k_automorph<4>, dim3(ewGrid(total)), AutArgs{out, in, g, m.count});
    checkLaunch(d, "automorph");
}

// ---- scratch owned by the device (per lane, grow-only) ----
// A lane's scratch is reused by every prim on that lane (stream-ordered).  A
// buffer that has to grow is retired, not freed: work already queued (or a
// captured graph) may still address it; retired buffers are released by
// sfp_destroy.  Returns nullptr (and records the error) when HBM is exhausted.
static u64* scratch(sfp_dev* d, size_t words) {
    std::lock_guard<std::mutex> g(d->scrMu);
    const int l = d->cur;
    if (d->scrWords[l] >= words) return d->scr[l];
    const size_t grow = std::max(words, d->scrWords[l] + d->scrWords[l] / 2);
    u64* p = nullptr;
    if (hipMalloc((void**)&p, grow * 8) != hipSuccess) {
        hipGetLastError();
        p = nullptr;
        if (hipMalloc((void**)&p, words * 8) != hipSuccess) {
            record(d, "scratch allocation", hipErrorOutOfMemory);
            return nullptr;
        }
        d->scrWords[l] = words;
    } else {
        d->scrWords[l] = grow;
    }
    if (d->scr[l]) d->retired.push_back(d->scr[l]);
    d->scr[l] = p;
    return p;
}

void sfp_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t ell, const uint64_t* qlinv,
                 uint32_t npoly, size_t inStride, size_t outStride) {
    sfp_rescale_ext(d, out, in, ell, ell - 1, qlinv, npoly, inStride, outStride);
}

// (in_p,i - lift(INTT(in_p,last))) * qlinv_i for both polys: INTT of the two
// dropped rows, then one NTT launch pair that lifts them to every remaining
// prime and applies the subtract-multiply in its last pass.
// Rescale of in * w: w = mulRows (elementwise, ell rows shared by the polys),
// w = mulK (host array of ell per-row residues) or w = 1.  The dropped row is
// multiplied on its INTT's load, the kept rows in the epilogue.
static void rescaleCore(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t ell, uint32_t dropPrime,
                        const uint64_t* qlinv, uint32_t npoly, size_t inStride, size_t outStride,
                        const uint64_t* mulRows, const uint64_t* mulK) {
    const uint32_t n = d->n;
    const uint32_t cnt = ell - 1;
    if (cnt > SFP_MAX_LIMBS || ell < 2) {
        record(d, "rescale (limb count)", hipErrorInvalidValue);
        return;
    }
    u64* last = scratch(d, (size_t)npoly * n + (size_t)npoly * cnt * n);
    if (!last) return;
    u64* tmp = last + (size_t)npoly * n;
    RowGroup A = rowsOf(npoly, 1, sfp_limbs{1, 0, dropPrime, 0});
    A.src = RowPtr{in + (size_t)cnt * n, (long long)inStride, 0};
    A.dst = RowPtr{last, (long long)n, 0};
    // per-call multipliers: content-cached device constants (a miss uploads
    // synchronously after draining every lane, so any lane may read a hit);
    // the sort's scalars repeat every call, so after the first sort this
    // launches no upload copy at all
    u64 mk[2 * SFP_MAX_LIMBS + 2];
    const u64* dmk = nullptr;
    if (mulRows) A.pre = RowPtr{mulRows + (size_t)cnt * n, 0, 0};
    if (mulK) {
        for (uint32_t i = 0; i < cnt; ++i) {
            mk[i] = mulK[i];
            mk[cnt + i] = sf_shoup_precomp(mulK[i], d->hbar[i].q);
        }
        mk[2 * cnt] = mulK[cnt];
        mk[2 * cnt + 1] = sf_shoup_precomp(mulK[cnt], d->hbar[dropPrime].q);
        dmk = devConst(d, mk, 2 * cnt + 2);
        A.preK = dmk + 2 * cnt;
        A.preKS = dmk + 2 * cnt + 1;
    }
    // the dropped row's inverse COL pass runs in the lift pass's prologue
    // (icol) where that pass has one: one dependent launch fewer per rescale
    const bool icol = icolPath(d, npoly * cnt);
    nttRows(d, A, 1, icol ? 1 : 3);
    RowGroup B = rowsOf(npoly, cnt, sfp_limbs{cnt, cnt, 0, 0});
    B.src = RowPtr{last, (long long)n, 0};
    B.lift = 1;
    B.liftPrime = dropPrime;
    if (icol) {
        B.icol = 1;
        B.iTw = d->ipsi;
        B.iTwS = d->ipsiS;
        B.iTwD = d->ipsiD;
    }
    B.dst = RowPtr{tmp, (long long)cnt * n, (long long)n};
    B.epi = 1;
    B.ein = RowPtr{in, (long long)inStride, (long long)n};
    B.eout = RowPtr{out, (long long)outStride, (long long)n};
    const u64 ql = d->hbar[dropPrime].q;
    u64 kS[SFP_MAX_LIMBS], lsub[SFP_MAX_LIMBS];
    for (uint32_t i = 0; i < cnt; ++i) {
        const u64 q = d->hbar[i].q;
        kS[i] = sf_shoup_precomp(qlinv[i], q);
        lsub[i] = ql % q;
    }
    B.k = devConst(d, qlinv, cnt);
    B.kS = devConst(d, kS, cnt);
    B.liftSub = devConst(d, lsub, cnt);
    if (mulRows) B.emul = RowPtr{mulRows, 0, (long long)n};
    if (mulK) {
        B.emK = dmk;
        B.emKS = dmk + cnt;
    }
    nttRows(d, B, 0);
}

void sfp_rescale_ext(sfp_dev* d, uint64_t* out, const uint64_t* in, uint32_t ell, uint32_t dropPrime,
                     const uint64_t* qlinv, uint32_t npoly, size_t inStride, size_t outStride) {
    rescaleCore(d, out, in, ell, dropPrime, qlinv, npoly, inStride, outStride, nullptr, nullptr);
}

void sfp_mul_const_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* k, uint32_t ell,
                           const uint64_t* qlinv, uint32_t npoly, size_t inStride, size_t outStride) {
    rescaleCore(d, out, in, ell, ell - 1, qlinv, npoly, inStride, outStride, nullptr, k);
}

void sfp_mul_rescale(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* m, uint32_t ell,
                     const uint64_t* qlinv, uint32_t npoly, size_t inStride, size_t outStride) {
    rescaleCore(d, out, in, ell, ell - 1, qlinv, npoly, inStride, outStride, m, nullptr);
}

// ---- base conversion / key switching ----
sfp_conv* sfp_upload_conv(sfp_dev* d, uint32_t ns, const uint32_t* src, uint32_t nt,
                          const uint32_t* dst, const uint32_t* drow, const uint64_t* inv,
                          const uint64_t* mod) {
    if (ns > (uint32_t)kMaxConvSrc) {
        record(d, "upload_conv (too many source primes)", hipErrorInvalidValue);
        return nullptr;
    }
    auto* c = new sfp_conv;
    c->ns = ns;
    c->nt = nt;
    c->hsrc.assign(src, src + ns);
    c->hdst.assign(dst, dst + nt);
    c->hinv.assign(inv, inv + ns);
    c->hmod.assign(mod, mod + (size_t)ns * nt);
    for (uint32_t t = 0; t < nt; ++t) c->hrow.push_back(drow ? drow[t] : t);
    // every device table is checked: a failed allocation must surface as an
    // error here, not as a conversion kernel writing through a null pointer
    bool ok = true;
    auto dmalloc = [&](auto*& dp, size_t bytes) {
        if (!ok) return;
        if (hipMalloc((void**)&dp, bytes + 8) != hipSuccess) {
            hipGetLastError();
            dp = nullptr;
            ok = false;
        }
    };
    dmalloc(c->src, ns * 4);
    dmalloc(c->dst, nt * 4);
    dmalloc(c->inv, ns * 8);
    dmalloc(c->mod, (size_t)ns * nt * 8);
    dmalloc(c->drow, nt * 4);
    dmalloc(c->sprod, nt * 8);
    if (!ok) {
        record(d, "upload_conv allocation", hipErrorOutOfMemory);
        sfp_free_conv(d, c);
        return nullptr;
    }
    std::vector<uint32_t> rows(nt);
    for (uint32_t t = 0; t < nt; ++t) rows[t] = drow ? drow[t] : t;
    hostToDev(d, c->drow, rows.data(), nt * 4);
    hostToDev(d, c->src, src, ns * 4);
    hostToDev(d, c->dst, dst, nt * 4);
    hostToDev(d, c->inv, inv, ns * 8);
    hostToDev(d, c->mod, mod, (size_t)ns * nt * 8);
    std::vector<u64> sp(nt);
    for (uint32_t t = 0; t < nt; ++t) {
        const sf_barrett& B = d->hbar[dst[t]];
        u64 r = 1;
        for (uint32_t i = 0; i < ns; ++i) r = sf_mul(r, d->hbar[src[i]].q % B.q, &B);
        sp[t] = r;
    }
    hostToDev(d, c->sprod, sp.data(), nt * 8);
    // FP64 form: FP64 / integer target split, multipliers over the FP64
    // targets, the 60-bit sources' second multiplier (mod * 2^30 mod p)
    for (uint32_t t = 0; t < nt; ++t)
        (d->hbar[dst[t]].q < kFpPrimeBound ? c->hFpT : c->hIntT).push_back(t);
    std::vector<uint32_t> bigs;
    for (uint32_t i = 0; i < ns; ++i)
        if (d->hbar[src[i]].q >= kFpPrimeBound) bigs.push_back(i);
    c->nbig = (uint32_t)bigs.size();
    c->fpOk = bigs.size() <= (size_t)kMaxConvBig;
    const size_t nf = c->hFpT.size();
    std::vector<double> invD(ns), invQ(ns), vD(ns * nf + 1), vQ(ns * nf + 1), hD(kMaxConvBig * nf + 1, 0.0),
        hQ(kMaxConvBig * nf + 1, 0.0);
    for (uint32_t i = 0; i < ns; ++i) {
        invD[i] = (double)inv[i];
        invQ[i] = (double)inv[i] / (double)d->hbar[src[i]].q;
        for (size_t k = 0; k < nf; ++k) {
            const uint32_t t = c->hFpT[k];
            const u64 m = mod[(size_t)i * nt + t];
            vD[i * nf + k] = (double)m;
            vQ[i * nf + k] = (double)m / (double)d->hbar[dst[t]].q;
        }
    }
    for (size_t b = 0; b < bigs.size() && b < (size_t)kMaxConvBig; ++b)
        for (size_t k = 0; k < nf; ++k) {
            const uint32_t t = c->hFpT[k];
            const u64 p = d->hbar[dst[t]].q;
            const u64 m = (u64)(((unsigned __int128)mod[(size_t)bigs[b] * nt + t] << 30) % p);
            hD[b * nf + k] = (double)m;
            hQ[b * nf + k] = (double)m / (double)p;
        }
    auto up = [&](auto*& dp, const auto& v) {
        dmalloc(dp, v.size() * sizeof(v[0]));
        if (ok) hostToDev(d, dp, v.data(), v.size() * sizeof(v[0]));
    };
    for (uint32_t t = 0; t < nt; ++t) c->hAll.push_back(t);
    up(c->fpT, c->hFpT);
    up(c->intT, c->hIntT);
    up(c->allT, c->hAll);
    up(c->invD, invD);
    up(c->invQ, invQ);
    up(c->vD, vD);
    up(c->vQ, vQ);
    up(c->hD, hD);
    up(c->hQ, hQ);
    // a ModDown table (every source FP64, target t on prime t and row t): the
    // fused COL pass's multipliers over every target (k_moddown_col)
    bool mdOk = c->nbig == 0;
    for (uint32_t t = 0; t < nt && mdOk; ++t) mdOk = dst[t] == t && rows[t] == t;
    if (mdOk) {
        std::vector<double> mD((size_t)ns * nt), mQ((size_t)ns * nt), spD(nt), spQ(nt);
        for (uint32_t t = 0; t < nt; ++t) {
            const double q = (double)d->hbar[t].q;
            for (uint32_t i = 0; i < ns; ++i) {
                mD[(size_t)i * nt + t] = (double)mod[(size_t)i * nt + t];
                mQ[(size_t)i * nt + t] = mD[(size_t)i * nt + t] / q;
            }
            spD[t] = (double)sp[t];
            spQ[t] = spD[t] / q;
        }
        up(c->mdD, mD);
        up(c->mdQ, mQ);
        up(c->mdSpD, spD);
        up(c->mdSpQ, spQ);
        c->mdState = ok ? 1 : -1;
    } else {
        c->mdState = -1;
    }
    if (!ok) {
        record(d, "upload_conv allocation", hipErrorOutOfMemory);
        sfp_free_conv(d, c);
        return nullptr;
    }
    return c;
}

void sfp_free_conv(sfp_dev* d, sfp_conv* c) {
    if (!c) return;
    syncAll(d);
    for (auto it = d->plans.begin(); it != d->plans.end();) {  // the levels' fused-ModUp plans that use c
        ModUpPlan* P = it->second;
        if (it->first == c || (P && std::find(P->convs.begin(), P->convs.end(), c) != P->convs.end())) {
            if (P) freePlan(P);
            it = d->plans.erase(it);
        } else {
            ++it;
        }
    }
    hipFree(c->src);
    hipFree(c->dst);
    hipFree(c->inv);
    hipFree(c->mod);
    hipFree(c->sprod);
    hipFree(c->drow);
    hipFree(c->fpT);
    hipFree(c->intT);
    hipFree(c->allT);
    for (double* x : {c->invD, c->invQ, c->vD, c->vQ, c->hD, c->hQ, c->mdD, c->mdQ, c->mdSpD, c->mdSpQ}) hipFree(x);
    delete c;
}

static ConvJob convJob(const sfp_conv* c, u64* dst, const u64* src, uint32_t ntUse, int centered) {
    ConvJob j;
    j.src = src;
    j.dst = dst;
    j.sidx = c->src;
    j.didx = c->dst;
    j.drow = c->drow;
    j.inv = c->inv;
    j.mod = c->mod;
    j.sprod = c->sprod;
    j.fpT = c->fpT;
    j.intT = c->intT;
    j.invD = c->invD;
    j.invQ = c->invQ;
    j.vD = c->vD;
    j.vQ = c->vQ;
    j.hD = c->hD;
    j.hQ = c->hQ;
    j.ns = c->ns;
    j.nt = c->nt;
    j.ntUse = ntUse;
    j.centered = (uint32_t)centered;
    // the FP64 / integer target lists are ascending: their first entries are
    // the targets below ntUse
    j.nFp = (uint32_t)(std::lower_bound(c->hFpT.begin(), c->hFpT.end(), ntUse) - c->hFpT.begin());
    j.nInt = (uint32_t)(std::lower_bound(c->hIntT.begin(), c->hIntT.end(), ntUse) - c->hIntT.begin());
    j.nFpAll = (uint32_t)c->hFpT.size();
    j.nbig = c->nbig;
    if (!c->fpOk) {  // more 60-bit sources than the FP64 form splits: integer targets only
        j.nFp = 0;
        j.intT = c->allT;
        j.nInt = ntUse;
    }
    return j;
}


static void convLaunch(sfp_dev* d, const ConvJobs& J, uint32_t njobs, bool fpOk) {
    if (!njobs) return;
    uint32_t maxT = 0, maxS = 0, maxZ = 0;
    double bytes = 0;
    for (uint32_t k = 0; k < njobs; ++k) {
        const ConvJob& j = J.j[k];
        maxT = std::max(maxT, j.ntUse);
        maxS = std::max(maxS, j.ns);
        maxZ = std::max(maxZ, (j.nFp + kConvChunk - 1) / kConvChunk +
                                  (convIntFolded(j.nbig, j.nFp, j.nInt) ? 0 : (j.nInt + kConvChunk - 1) / kConvChunk));
        bytes += 8.0 * d->n * (j.ns + j.ntUse);
    }
    // the block-cooperative kernel (k_convf) runs every job: FP64 targets in
    // FP64, the rest -- or, for tables with more 60-bit sources than it splits,
    // every target (convJob) -- on its integer blocks.  k_conv (one thread per
    // coefficient pair, 255 VGPRs, one wave per SIMD) only serves
    // SFHE_NTT_FP=0.
    (void)fpOk;
    const bool fp = nttFp() != 0;
    const uint32_t gz = fp ? maxZ : (maxT + kConvChunk - 1) / kConvChunk;
    if (!gz) return;
    const dim3 g(fp ? d->n / kConvCoefs : d->n / (2 * kThreads), njobs, gz);
    timedLaunch(d, SFP_FAM_CONV, bytes, [&] {
        // NS = 13 (ModDown's K P-rows, ModUp digits of <= 13 primes) sizes the
        // LDS for 6 blocks per CU instead of 5 (the loops keep their guards)
        ConvKern k = (fp && maxS <= 13) ? k_convf<13> : (fp && maxS <= 16) ? k_convf<16>
                     : fp                ? k_convf<kMaxConvSrc>
                                         : k_conv;
        StackRec r;
        r.go = [=](hipStream_t s_) { hipLaunchKernelGGL(k, g, dim3(kThreads), 0, s_, J, d->bar, d->qinvD, d->logn); };
        if (d->stackOn) {
            auto P = std::make_shared<ConvPay>();
            P->J = J;
            P->njobs = njobs;
            P->g = g;
            P->k = k;
            r.cls = STK_CONV;
            r.key = stkKey((const void*)k, g.x, 0);
            r.pay = std::move(P);
        }
        issueRec(d, std::move(r));
    });
    checkLaunch(d, "conv");
}

void sfp_conv_apply(sfp_dev* d, uint64_t* dst, const uint64_t* src, const sfp_conv* c) {
    ConvJobs J;
    J.j[0] = convJob(c, dst, src, c->nt, 0);
    convLaunch(d, J, 1, c->fpOk);
}

void sfp_conv_apply_centered(sfp_dev* d, uint64_t* dst, const uint64_t* src, const sfp_conv* c,
                             uint32_t ntUse) {
    if (!c || !ntUse) return;
    ConvJobs J;
    J.j[0] = convJob(c, dst, src, std::min(ntUse, c->nt), 1);
    convLaunch(d, J, 1, c->fpOk);
}

// ModUp with its conversion fused into the forward COL pass (VERDICT r4
// item 3): the INTT's last pass leaves y_s = [x_s * shat_s^-1]_{q_s} (its n^-1
// times the conversion's source factor, per row) with FP64 rows stored as
// doubles, and the COL pass of target row i of digit p computes its tile as
// sum_s y_s * [shat_s]_{q_i} mod q_i from the digit's source tiles -- the
// extended limbs are never written before their NTT, and k_convf's launch is
// gone.  Same integers as k_convf + the plain COL pass (canonical residues).
// Per level (keyed by its digit-0 table): the INTT's per-row constants and
// the multipliers indexed by ext row.  Eligible where the FP64 form applies
// to every source but q_0 (60-bit: split in two 30-bit halves) and the COL
// pass runs LE = 2 (the defaults); otherwise the unfused launches run.
static bool modupFuseOn() {  // SFHE_MODUP_FUSE=0: k_convf + the plain COL pass (A/B)
    static const bool on = [] {
        const char* v = std::getenv("SFHE_MODUP_FUSE");
        return !v || *v != '0';
    }();
    return on;
}
static const ModUpPlan* modupPlan(sfp_dev* d, const sfp_conv* const* convs, uint32_t ell, uint32_t K,
                                  uint32_t alpha) {
    if (!modupFuseOn() || !nttFp() || d->n <= (uint32_t)kNttTile || nttSmallLe() != 2 || nttSmallTile() != 1024 ||
        (nttLe() != 0 && nttLe() != 2))
        return nullptr;
    auto it = d->plans.find(convs[0]);
    if (it != d->plans.end()) return it->second;
    const uint32_t beta = (ell + alpha - 1) / alpha, rows = ell + K;
    // eligibility: digit j's sources are rows j alpha + s; only q_0 (digit 0, s = 0) is 60-bit
    bool ok = true;
    bool big = false;
    for (uint32_t j = 0; j < beta && ok; ++j) {
        const sfp_conv* c = convs[j];
        ok = c->ns == std::min(alpha, ell - j * alpha);
        for (uint32_t sI = 0; sI < c->ns && ok; ++sI) {
            ok = c->hsrc[sI] == j * alpha + sI;
            if (d->hbar[c->hsrc[sI]].q >= kFpPrimeBound) {
                ok = ok && j == 0 && sI == 0;
                big = true;
            }
        }
        for (uint32_t t = 0; t < c->nt && ok; ++t) ok = c->hrow[t] < rows;
    }
    if (!ok) {
        d->plans[convs[0]] = nullptr;
        return nullptr;
    }
    auto* P = new ModUpPlan;
    P->ell = ell;
    P->rows = rows;
    P->big = big;
    P->convs.assign(convs, convs + beta);
    std::vector<u64> pk(ell), pks(ell), mI((size_t)beta * alpha * rows, 0);
    std::vector<double> pd(ell), pq(ell), mD((size_t)beta * alpha * rows, 0.0), mQ((size_t)beta * alpha * rows, 0.0),
        hD(rows, 0.0), hQ(rows, 0.0);
    for (uint32_t j = 0; j < beta; ++j) {
        const sfp_conv* c = convs[j];
        for (uint32_t sI = 0; sI < c->ns; ++sI) {
            const uint32_t r = j * alpha + sI, pr = c->hsrc[sI];
            const sf_barrett& B = d->hbar[pr];
            const u64 k = sf_mul(c->hinv[sI] % B.q, d->hninv[pr] % B.q, &B);
            pk[r] = k;
            pks[r] = sf_shoup_precomp(k, B.q);
            pd[r] = (double)k;
            pq[r] = (double)k / (double)B.q;
            for (uint32_t t = 0; t < c->nt; ++t) {
                const uint32_t row = c->hrow[t];
                const u64 p = d->hbar[c->hdst[t]].q, m = c->hmod[(size_t)sI * c->nt + t];
                const size_t o = ((size_t)j * alpha + sI) * rows + row;
                mI[o] = m;
                mD[o] = (double)m;
                mQ[o] = (double)m / (double)p;
                if (big && j == 0 && sI == 0) {
                    const u64 h = (u64)(((unsigned __int128)m << 30) % p);
                    hD[row] = (double)h;
                    hQ[row] = (double)h / (double)p;
                }
            }
        }
    }
    bool mok = true;
    auto up = [&](auto*& dp, const auto& v) {
        if (!mok) return;
        if (hipMalloc((void**)&dp, v.size() * sizeof(v[0]) + 8) != hipSuccess) {
            hipGetLastError();
            dp = nullptr;
            mok = false;
            return;
        }
        hostToDev(d, dp, v.data(), v.size() * sizeof(v[0]));
    };
    up(P->postK, pk);
    up(P->postKS, pks);
    up(P->postD, pd);
    up(P->postQ, pq);
    up(P->mD, mD);
    up(P->mQ, mQ);
    up(P->mI, mI);
    up(P->hD, hD);
    up(P->hQ, hQ);
    if (!mok) {
        record(d, "modup plan allocation", hipErrorOutOfMemory);
        freePlan(P);
        return nullptr;
    }
    d->plans[convs[0]] = P;
    return P;
}
void sfp_modup_prepare(sfp_dev* d, const sfp_conv* const* convs, uint32_t ell, uint32_t K, uint32_t alpha) {
    const uint32_t beta = (ell + alpha - 1) / alpha;
    if (!convs || d->capture || beta > (uint32_t)kMaxConvJobs || ell + K > SFP_MAX_LIMBS) return;
    modupPlan(d, convs, ell, K, alpha);
}
static void planInto(const ModUpPlan* P, RowGroup& A, RowGroup& B, const u64* y) {
    A.postK = P->postK;
    A.postKS = P->postKS;
    A.postD = P->postD;
    A.postQ = P->postQ;
    B.cy = y;
    B.cmD = P->mD;
    B.cmQ = P->mQ;
    B.cmI = P->mI;
    B.chD = P->hD;
    B.chQ = P->hQ;
    B.cRows = P->rows;
    B.cBig = P->big ? 1u : 0u;
}

void sfp_modup(sfp_dev* d, uint64_t* ext, const uint64_t* in, uint32_t ell, uint32_t K,
               uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, uint64_t* scr) {
    const uint32_t n = d->n;
    const uint32_t beta = (ell + alpha - 1) / alpha;
    const long long stride = (long long)(ell + K) * n;
    if (beta > (uint32_t)kMaxConvJobs || ell + K > SFP_MAX_LIMBS) {
        record(d, "modup (too many digits / limbs)", hipErrorInvalidValue);
        return;
    }
    // INTT of every input row; the raw rows go to their digit's ext block
    RowGroup A = rowsOf(1, ell, sfp_limbs{ell, ell, 0, 0});
    A.src = RowPtr{in, 0, (long long)n};
    A.dst = RowPtr{scr, 0, (long long)n};
    A.copy = RowPtr{ext, stride, (long long)n};
    A.copyByAlpha = 1;
    A.alpha = alpha;
    RowGroup B = rowsOf(beta, ell + K, sfp_limbs{ell + K, ell, Lq, 0});
    B.src = B.dst = RowPtr{ext, stride, (long long)n};
    B.skipEll = ell;
    B.alpha = alpha;
    const ModUpPlan* P = modupPlan(d, convs, ell, K, alpha);
    if (P) planInto(P, A, B, scr);
    nttRows(d, A, 1);
    if (!P) {  // every digit's conversion in one launch
        ConvJobs J;
        bool fpOk = true;
        for (uint32_t j = 0; j < beta; ++j) {
            J.j[j] = convJob(convs[j], ext + j * stride, scr + (size_t)j * alpha * n, convs[j]->nt, 0);
            fpOk = fpOk && convs[j]->fpOk;
        }
        convLaunch(d, J, beta, fpOk);
    }
    // NTT of every converted row (digit-own rows skipped)
    nttRows(d, B, 0);
}

static bool ksFuse() {  // SFHE_KS_FUSE=0: the unfused sequences (A/B)
    static const bool on = [] {
        const char* v = std::getenv("SFHE_KS_FUSE");
        return !v || *v != '0';
    }();
    return on;
}

// The fused ModUp + key inner product (sfp_modup_inner / sfp_mult_relin_rescale):
// INTT of the input (in, or in (.) inMul: a tensor's d2 = a1 b1 formed in the
// first pass), the digits' conversions, the forward COL pass, then k_ntt_ks.
// T[4] (a0, a1, b0, b1) non-null: the fold rows are the tensor's d0 / d1.
static void modupInnerCore(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* in, const uint64_t* inMul,
                           uint32_t ell, uint32_t K, uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs,
                           const uint64_t* key, const uint64_t* fold0, const uint64_t* fold1,
                           const uint64_t* const* T, uint64_t foldK, int accum, uint32_t invFrom, uint64_t* ext,
                           uint64_t* scr, int phases = 3) {
    const uint32_t n = d->n;
    const uint32_t beta = (ell + alpha - 1) / alpha;
    const long long stride = (long long)(ell + K) * n;
    if (phases & 1) {
    // INTT of every input row (the digits' own rows are read from `in` by the fused pass)
    RowGroup A = rowsOf(1, ell, sfp_limbs{ell, ell, 0, 0});
    A.src = RowPtr{in, 0, (long long)n};
    A.dst = RowPtr{scr, 0, (long long)n};
    if (inMul) A.pre = RowPtr{inMul, 0, (long long)n};
    RowGroup B = rowsOf(beta, ell + K, sfp_limbs{ell + K, ell, Lq, 0});
    B.src = B.dst = RowPtr{ext, stride, (long long)n};
    B.skipEll = ell;
    B.alpha = alpha;
    const ModUpPlan* P = modupPlan(d, convs, ell, K, alpha);
    if (P) planInto(P, A, B, scr);
    nttRows(d, A, 1);
    if (!P) {
        ConvJobs J;
        bool fpOk = true;
        for (uint32_t j = 0; j < beta; ++j) {
            J.j[j] = convJob(convs[j], ext + j * stride, scr + (size_t)j * alpha * n, convs[j]->nt, 0);
            fpOk = fpOk && convs[j]->fpOk;
        }
        convLaunch(d, J, beta, fpOk);
    }
    // the forward COL pass of every converted row (with the conversion in
    // its prologue where a plan applies); the ROW pass runs fused below
    nttRows(d, B, 0, 1);
    }
    if (!(phases & 2)) return;
    KsArgs a;
    std::memset(&a, 0, sizeof a);
    a.in = in;
    a.inMul = inMul;
    a.ext = ext;
    a.extStride = stride;
    a.key = key;
    a.keyRows = d->kg.rows ? d->kg.rows : Lq + K;  // (a sliced key: sfp_set_key_geom)
    a.keyQ = d->kg.rows ? d->kg.pstart : Lq;
    a.acc0 = acc0;
    a.acc1 = acc1;
    a.fold0 = fold0;
    a.fold1 = fold1;
    if (T) {
        a.fa0 = T[0];
        a.fa1 = T[1];
        a.fb0 = T[2];
        a.fb1 = T[3];
    }
    a.foldK = foldK;
    a.ell = ell;
    a.Lq = Lq;
    a.alpha = alpha;
    a.beta = beta;
    a.accum = accum;
    a.invFrom = invFrom;
    a.itw = d->ipsi;
    a.itwS = d->ipsiS;
    a.itwD = d->ipsiD;
    const uint32_t rows = ell + K;
    const size_t total = (size_t)rows * n;
    const bool t1k = rows <= 64 && n <= 1024u * 128u;
    timedLaunch(d, SFP_FAM_NTTKS, 8.0 * total * (3.0 * beta + (accum ? 4.0 : 2.0)), [&] {
        ArgSet<KsArgs, 1> AS;
        AS.a[0] = a;
        AS.start[0] = 0;
        AS.inter = 0;
        const int fp = nttFp();
        const dim3 g(n / (t1k ? 1024u : (uint32_t)kNttTile), rows);
        const int threads = (t1k ? 1024 : kNttTile) >> 2;
        auto k1 = t1k ? k_ntt_ks<2, 1024> : k_ntt_ks<2, kNttTile>;
        StackRec r;
        r.go = [=](hipStream_t s_) {
            hipLaunchKernelGGL(k1, g, dim3(threads), 0, s_, AS, d->bar, d->psi, d->psiS, d->logn, d->psiD, d->qinvD,
                               fp, d->rowD);
        };
        if (d->stackOn) {
            auto P = std::make_shared<KsPay>();
            P->a = a;
            P->rows = rows;
            P->g = g;
            P->threads = threads;
            P->useFp = fp;
            P->k2 = t1k ? k_ntt_ks<2, 1024, 2> : k_ntt_ks<2, kNttTile, 2>;
            P->k4 = t1k ? k_ntt_ks<2, 1024, 4> : k_ntt_ks<2, kNttTile, 4>;
            P->k8 = t1k ? k_ntt_ks<2, 1024, 8> : k_ntt_ks<2, kNttTile, 8>;
            r.cls = STK_KS;
            r.key = stkKey((const void*)k1, g.x, (uint32_t)threads);
            r.pay = std::move(P);
        }
        issueRec(d, std::move(r));
    });
    checkLaunch(d, "ntt_ks");
}

int sfp_modup_inner_phase(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* in, uint32_t ell, uint32_t K,
                          uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key,
                          const uint64_t* fold0, const uint64_t* fold1, uint64_t foldK, int accum, uint32_t invFrom,
                          uint64_t* ext, uint64_t* scr, int phases) {
    const uint32_t beta = (ell + alpha - 1) / alpha;
    if (!ksFuse() || d->n <= (uint32_t)kNttTile) return -1;  // the caller runs sfp_modup + sfp_ks_inner*
    if (!phases) return 0;
    if (beta > (uint32_t)kMaxConvJobs || ell + K > SFP_MAX_LIMBS || (fold0 && (!fold1 || ell < 1))) {
        record(d, "modup_inner (too many digits / limbs)", hipErrorInvalidValue);
        return 0;
    }
    modupInnerCore(d, acc0, acc1, in, nullptr, ell, K, Lq, alpha, convs, key, fold0, fold1, nullptr, foldK, accum,
                   invFrom, ext, scr, phases);
    return 0;
}

int sfp_modup_inner(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* in, uint32_t ell, uint32_t K,
                    uint32_t Lq, uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key,
                    const uint64_t* fold0, const uint64_t* fold1, uint64_t foldK, int accum, uint32_t invFrom,
                    uint64_t* ext, uint64_t* scr) {
    return sfp_modup_inner_phase(d, acc0, acc1, in, ell, K, Lq, alpha, convs, key, fold0, fold1, foldK, accum,
                                 invFrom, ext, scr, 3);
}

void sfp_ks_inner(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                  size_t extStride, const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K,
                  uint32_t Lq) {
    sfp_ks_inner_fold(d, acc0, acc1, ext, extStride, key, beta, ell, K, Lq, nullptr, nullptr, 0);
}

void sfp_ks_inner_fold(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext,
                       size_t extStride, const uint64_t* key, uint32_t beta, uint32_t ell,
                       uint32_t K, uint32_t Lq, const uint64_t* fold0, const uint64_t* fold1,
                       uint64_t foldK) {
    const uint32_t keyQ0 = d->kg.rows ? d->kg.pstart : Lq, keyRows0 = d->kg.rows ? d->kg.rows : Lq + K;
    const size_t total = (size_t)(ell + K) * d->n;
    if (fold0 && (!fold1 || ell < 1)) {
        record(d, "ks_inner_fold", hipErrorInvalidValue);
        return;
    }
    // reads beta ext rows + 2*beta key rows, writes 2 accumulator rows, per limb
    timedLaunch(d, SFP_FAM_KSINNER, 8.0 * total * (3.0 * beta + 2.0), [&] {
        issueY<KsInnerArgs>(d, k_ks_inner<1>, k_ks_inner<2>, k_ks_inner<4>, dim3(ewGrid(total / 2)),
                                KsInnerArgs{acc0, acc1, ext, extStride, key, beta, sfp_limbs{ell + K, ell, Lq, 0, 1}, keyQ0, keyRows0, fold0, fold1, foldK, 0, (const u64*)nullptr, d->kg, 0u});
    });
    checkLaunch(d, "ks_inner");
}

void sfp_ks_inner_aut(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext, size_t extStride,
                      const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K, uint32_t Lq, uint32_t gal) {
    const uint32_t keyQ0 = d->kg.rows ? d->kg.pstart : Lq, keyRows0 = d->kg.rows ? d->kg.rows : Lq + K;
    const size_t total = (size_t)(ell + K) * d->n;
    timedLaunch(d, SFP_FAM_KSINNER, 8.0 * total * (3.0 * beta + 2.0), [&] {
        issueY<KsInnerArgs>(d, k_ks_inner<1>, k_ks_inner<2>, k_ks_inner<4>, dim3(ewGrid(total / 2)),
                                KsInnerArgs{acc0, acc1, ext, extStride, key, beta, sfp_limbs{ell + K, ell, Lq, 0, 1}, keyQ0, keyRows0, (const u64*)nullptr, (const u64*)nullptr, (u64)0, 0, (const u64*)nullptr, d->kg, gal});
    });
    checkLaunch(d, "ks_inner_aut");
}

void sfp_ks_inner_acc(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext, size_t extStride,
                      const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K, uint32_t Lq) {
    const uint32_t keyQ0 = d->kg.rows ? d->kg.pstart : Lq, keyRows0 = d->kg.rows ? d->kg.rows : Lq + K;
    const size_t total = (size_t)(ell + K) * d->n;
    // reads beta ext rows + 2*beta key rows + 2 accumulator rows, writes 2, per limb
    timedLaunch(d, SFP_FAM_KSINNER, 8.0 * total * (3.0 * beta + 4.0), [&] {
        issueY<KsInnerArgs>(d, k_ks_inner<1>, k_ks_inner<2>, k_ks_inner<4>, dim3(ewGrid(total / 2)),
                                KsInnerArgs{acc0, acc1, ext, extStride, key, beta, sfp_limbs{ell + K, ell, Lq, 0, 1}, keyQ0, keyRows0, (const u64*)nullptr, (const u64*)nullptr, (u64)0, 1, (const u64*)nullptr, d->kg, 0u});
    });
    checkLaunch(d, "ks_inner_acc");
}

void sfp_ks_inner_mul(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext, size_t extStride,
                      const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K, uint32_t Lq, const uint64_t* pm,
                      int accum) {
    sfp_ks_inner_mul_aut(d, acc0, acc1, ext, extStride, key, beta, ell, K, Lq, pm, accum, 0);
}

void sfp_ks_inner_mul_aut(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext, size_t extStride,
                          const uint64_t* key, uint32_t beta, uint32_t ell, uint32_t K, uint32_t Lq,
                          const uint64_t* pm, int accum, uint32_t gal) {
    const uint32_t keyQ0 = d->kg.rows ? d->kg.pstart : Lq, keyRows0 = d->kg.rows ? d->kg.rows : Lq + K;
    const size_t total = (size_t)(ell + K) * d->n;
    // reads beta ext rows + 2*beta key rows + the plaintext row (+ 2 accumulator rows), writes 2, per limb
    timedLaunch(d, SFP_FAM_KSINNER, 8.0 * total * (3.0 * beta + (accum ? 5.0 : 3.0)), [&] {
        issueY<KsInnerArgs>(d, k_ks_inner<1>, k_ks_inner<2>, k_ks_inner<4>, dim3(ewGrid(total / 2)),
                                KsInnerArgs{acc0, acc1, ext, extStride, key, beta, sfp_limbs{ell + K, ell, Lq, 0, 1}, keyQ0, keyRows0, (const u64*)nullptr, (const u64*)nullptr, (u64)0, accum, pm, d->kg, gal});
    });
    checkLaunch(d, "ks_inner_mul");
}

// The fused ModDown COL pass (k_moddown_col): ring 2^16 with the default NTT
// shape (LE 2, 1024-word small tiles), a ModDown table (every source FP64,
// target t on prime t; sfp_upload_conv), with the rescale its dropped prime
// FP64 too.  Returns the call's device table (constant arena), or null: the
// unfused launches run.  Off by default (SFHE_MODDOWN_COL=1 turns it on): A/B
// x2 on one box, the metric sort 40.0-40.3 ms fused at every level and
// 38.7-39.0 up to 16 target rows, against 38.7 unfused.
static bool moddownColOn() {
    static const bool on = [] {
        const char* v = std::getenv("SFHE_MODDOWN_COL");
        return v && *v == '1';
    }();
    return on;
}
// A (the INTT of the P rows, after the rescale's dropped row l) gets the
// conversion's factors in its last pass: row of prime p_i -> n^-1 (P/p_i)^-1,
// row l -> n^-1; its FP64 rows are stored as doubles.
static const MdColArgs* mdColArgs(sfp_dev* d, const sfp_conv* c, uint32_t targets, bool rs, uint32_t l, uint32_t Lq,
                                  const u64* pmod, const u64* lsub, u64 pinvl, RowGroup& A) {
    if (!moddownColOn() || !nttFp() || d->logn != 16 || nttSmallLe() != 2 || nttSmallTile() != 1024 ||
        (nttLe() != 0 && nttLe() != 2) || c->mdState != 1 || c->ns > (uint32_t)kMaxConvSrc)
        return nullptr;
    static const uint32_t maxT = [] {  // SFHE_MODDOWN_COL_MAXT: fused up to this many target rows (A/B)
        const char* v = std::getenv("SFHE_MODDOWN_COL_MAXT");
        return v ? (uint32_t)std::atoi(v) : 1024u;
    }();
    if (targets > maxT) return nullptr;
    if (targets > c->nt || (rs && (l >= c->nt || d->hbar[l].q >= kFpPrimeBound))) return nullptr;
    for (uint32_t i = 0; i < c->ns; ++i)
        if (c->hsrc[i] != Lq + i) return nullptr;  // (A's rows: the P primes in order)
    const uint32_t rows = c->ns + (rs ? 1u : 0u);
    u64 pk[SFP_MAX_LIMBS], pks[SFP_MAX_LIMBS];
    double pd[SFP_MAX_LIMBS], pq[SFP_MAX_LIMBS];
    for (uint32_t r = 0; r < rows; ++r) {
        const bool dropped = rs && r == 0;
        const uint32_t pr = dropped ? l : c->hsrc[r - (rs ? 1 : 0)];
        const sf_barrett& B = d->hbar[pr];
        const u64 k = dropped ? d->hninv[pr] % B.q : sf_mul(c->hinv[r - (rs ? 1 : 0)] % B.q, d->hninv[pr] % B.q, &B);
        pk[r] = k;
        pks[r] = sf_shoup_precomp(k, B.q);
        pd[r] = (double)k;
        pq[r] = (double)k / (double)B.q;
    }
    A.postK = devConst(d, pk, rows);
    A.postKS = devConst(d, pks, rows);
    A.postD = reinterpret_cast<const double*>(devConst(d, reinterpret_cast<const u64*>(pd), rows));
    A.postQ = reinterpret_cast<const double*>(devConst(d, reinterpret_cast<const u64*>(pq), rows));
    MdColArgs a;
    std::memset(&a, 0, sizeof a);
    a.sidx = c->src;
    a.invD = c->invD;
    a.invQ = c->invQ;
    a.mD = c->mdD;
    a.mQ = c->mdQ;
    a.mI = c->mod;
    a.sprod = c->sprod;
    a.spD = c->mdSpD;
    a.spQ = c->mdSpQ;
    a.ns = c->ns;
    a.nt = c->nt;
    a.l = l;
    a.rs = rs ? 1u : 0u;
    if (rs) {
        double pd[SFP_MAX_LIMBS], pq[SFP_MAX_LIMBS];
        for (uint32_t i = 0; i < l; ++i) {
            pd[i] = (double)pmod[i];
            pq[i] = (double)pmod[i] / (double)d->hbar[i].q;
        }
        a.pmod = devConst(d, pmod, l);
        a.lsub = devConst(d, lsub, l);
        a.pmD = reinterpret_cast<const double*>(devConst(d, reinterpret_cast<const u64*>(pd), l));
        a.pmQ = reinterpret_cast<const double*>(devConst(d, reinterpret_cast<const u64*>(pq), l));
        a.pinvl = pinvl;
    }
    static_assert(sizeof(MdColArgs) % 8 == 0, "MdColArgs in 8-byte words");
    return reinterpret_cast<const MdColArgs*>(devConst(d, reinterpret_cast<const u64*>(&a), sizeof a / 8));
}

void sfp_moddown2(sfp_dev* d, uint64_t* out0, uint64_t* out1, uint64_t* acc, size_t accStride,
                  uint32_t ell, uint32_t K, uint32_t Lq, const sfp_conv* c, const uint64_t* pinv,
                  int add0, int add1, uint64_t* scr, int rowDone) {
    const uint32_t n = d->n;
    if (ell > SFP_MAX_LIMBS) {
        record(d, "moddown (too many limbs)", hipErrorInvalidValue);
        return;
    }
    u64* pRows = acc + (size_t)ell * n;
    RowGroup A = rowsOf(2, K, sfp_limbs{K, 0, Lq, 0});
    A.src = A.dst = RowPtr{pRows, (long long)accStride, (long long)n};
    const MdColArgs* md = mdColArgs(d, c, ell, false, 0, Lq, nullptr, nullptr, 0, A);
    nttRows(d, A, 1, rowDone ? 2 : 3);
    if (!md) {
        ConvJobs J;
        J.j[0] = convJob(c, scr, pRows, ell, 1);
        J.j[1] = convJob(c, scr + (size_t)ell * n, pRows + accStride, ell, 1);
        convLaunch(d, J, 2, c->fpOk);
    }
    RowGroup B = rowsOf(2, ell, sfp_limbs{ell, ell, 0, 0});
    B.src = B.dst = RowPtr{scr, (long long)ell * n, (long long)n};
    if (md) {  // the conversion in the forward COL pass (k_moddown_col)
        B.md = md;
        B.copy = RowPtr{pRows, (long long)accStride, (long long)n};
        B.cRows = c->ns;  // (source rows per polynomial: graph byte accounting)
    }
    B.epi = 1;
    B.addMask = (add0 ? 1u : 0u) | (add1 ? 2u : 0u);
    B.ein = RowPtr{acc, (long long)accStride, (long long)n};
    B.eout = RowPtr{out0, (long long)(out1 - out0), (long long)n};
    u64 kS[SFP_MAX_LIMBS];
    for (uint32_t i = 0; i < ell; ++i) kS[i] = sf_shoup_precomp(pinv[i], d->hbar[i].q);
    B.k = devConst(d, pinv, ell);
    B.kS = devConst(d, kS, ell);
    nttRows(d, B, 0);
}

// The integer ModDown + rescale (tables with 60-bit sources) on the block-
// cooperative k_mdrsi; SFHE_MDRSI=0: the one-thread-per-pair k_conv_mdrs (A/B)
static bool mdrsiOn() {
    static const bool on = [] {
        const char* v = std::getenv("SFHE_MDRSI");
        return !v || *v != '0';
    }();
    return on;
}

// sfp_moddown_rescale; T[4] (a0, a1, b0, b1) non-null: d0 / d1 are the
// tensor of (a0, a1) and (b0, b1), formed in the final pass's epilogue
static void moddownRescaleCore(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* d0, const uint64_t* d1,
                               const uint64_t* const* T, uint64_t* acc, size_t accStride, uint32_t ell, uint32_t K,
                               uint32_t Lq, const sfp_conv* c, const uint64_t* pinv, const uint64_t* pmod,
                               const uint64_t* qlinv, uint64_t* scr, int rowDone) {
    const uint32_t n = d->n, l = ell - 1;
    if (ell < 2 || ell > SFP_MAX_LIMBS || !c || c->ns > (uint32_t)kMaxConvSrc || c->nt < ell ||
        !limbsOk(d, sfp_limbs{K + 1, 1, Lq, l}, "moddown_rescale")) {
        record(d, "moddown_rescale", hipErrorInvalidValue);
        return;
    }
    // INTT of rows [l, ell+K) of both accumulators: the dropped q row and the P rows
    RowGroup A = rowsOf(2, K + 1, sfp_limbs{K + 1, 1, Lq, l});
    A.src = A.dst = RowPtr{acc + (size_t)l * n, (long long)accStride, (long long)n};
    // conversion + the dropped row's lift
    MdrsArgs M;
    std::memset(&M, 0, sizeof M);  // (stacked launches compare it bytewise)
    for (int p = 0; p < 2; ++p) {
        const u64* ap = acc + (size_t)p * accStride;
        M.j[p] = MdrsJob{ap + (size_t)ell * n, ap, scr + (size_t)p * l * n};
    }
    u64 lsub[SFP_MAX_LIMBS], k1[SFP_MAX_LIMBS], k1S[SFP_MAX_LIMBS], k2S[SFP_MAX_LIMBS];
    const u64 ql = d->hbar[l].q;
    for (uint32_t i = 0; i < l; ++i) {
        const u64 q = d->hbar[i].q;
        lsub[i] = ql % q;
        k1[i] = (u64)((unsigned __int128)pinv[i] * qlinv[i] % q);  // (P q_l)^-1
        k1S[i] = sf_shoup_precomp(k1[i], q);
        k2S[i] = sf_shoup_precomp(qlinv[i], q);
    }
    const MdColArgs* md = mdColArgs(d, c, l, true, l, Lq, pmod, lsub, pinv[l], A);
    nttRows(d, A, 1, rowDone ? 2 : 3);
    if (!md) {
        M.sidx = c->src;
        M.inv = c->inv;
        M.mod = c->mod;
        M.sprod = c->sprod;
        M.pmod = devConst(d, pmod, l);
        M.lsub = devConst(d, lsub, l);
        M.pinvl = pinv[l];
        M.ns = c->ns;
        M.nt = c->nt;
        M.l = l;
        // FP64 form: every source (P row) and the dropped row's prime FP64
        const auto lpos = std::lower_bound(c->hFpT.begin(), c->hFpT.end(), l);
        const bool fp = nttFp() && c->fpOk && c->nbig == 0 && lpos != c->hFpT.end() && *lpos == l;
        uint32_t zc = (l + kConvChunk - 1) / kConvChunk;
        if (fp) {
            M.fpT = c->fpT;
            M.intT = c->intT;
            M.invD = c->invD;
            M.invQ = c->invQ;
            M.vD = c->vD;
            M.vQ = c->vQ;
            M.nFpAll = (uint32_t)c->hFpT.size();
            M.lD = c->vD + (lpos - c->hFpT.begin());
            M.lQ = c->vQ + (lpos - c->hFpT.begin());
            M.nFp = (uint32_t)(lpos - c->hFpT.begin());
            M.nInt = (uint32_t)(std::lower_bound(c->hIntT.begin(), c->hIntT.end(), l) - c->hIntT.begin());
            double pd[SFP_MAX_LIMBS], pq[SFP_MAX_LIMBS];
            for (uint32_t i = 0; i < l; ++i) {
                pd[i] = (double)pmod[i];
                pq[i] = (double)pmod[i] / (double)d->hbar[i].q;
            }
            M.pmodD = reinterpret_cast<const double*>(devConst(d, reinterpret_cast<const u64*>(pd), l));
            M.pmodQ = reinterpret_cast<const double*>(devConst(d, reinterpret_cast<const u64*>(pq), l));
            zc = (M.nFp + kConvChunk - 1) / kConvChunk +
             (mdrsIntFolded(false, M.nFp, M.nInt) ? 0 : (M.nInt + kConvChunk - 1) / kConvChunk);
        }
        // the dropped prime 60-bit, FP64 sources, every target below it an
        // integer row (scale-59 chains): the integer-l form of k_mdrsf
        const bool bigl = !fp && nttFp() && c->fpOk && c->nbig == 0 && d->hbar[l].q >= kFpPrimeBound &&
                          (c->hFpT.empty() || c->hFpT.front() > l);
        if (bigl) {
            M.intT = c->intT;
            M.invD = c->invD;
            M.invQ = c->invQ;
            M.nFp = 0;
            M.nFpAll = (uint32_t)c->hFpT.size();
            M.nInt = (uint32_t)(std::lower_bound(c->hIntT.begin(), c->hIntT.end(), l) - c->hIntT.begin());
            zc = (M.nInt + kConvChunk - 1) / kConvChunk;
        }
        const dim3 g((fp || bigl || mdrsiOn()) ? n / kConvCoefs : n / (2 * kThreads), 2, zc);
        timedLaunch(d, SFP_FAM_CONV, 8.0 * n * 2 * (K + 1 + l), [&] {
            // (fp: LDS for 6 blocks per CU at ns <= 13, as convLaunch)
            MdrsKern k = (bigl && c->ns <= 13) ? k_mdrsf<13, true>
                         : (bigl && c->ns <= 16) ? k_mdrsf<16, true>
                         : bigl                  ? k_mdrsf<kMaxConvSrc, true>
                         : (fp && c->ns <= 13)   ? k_mdrsf<13>
                         : (fp && c->ns <= 16)   ? k_mdrsf<16>
                         : fp                    ? k_mdrsf<kMaxConvSrc>
                         : !mdrsiOn()            ? k_conv_mdrs
                         : c->ns <= 16           ? k_mdrsi<16>
                                                 : k_mdrsi<kMaxConvSrc>;
            StackRec r;
            r.go = [=](hipStream_t s_) { hipLaunchKernelGGL(k, g, dim3(kThreads), 0, s_, M, d->bar, d->qinvD, d->logn); };
            if (d->stackOn) {
                auto P = std::make_shared<MdrsPay>();
                P->M = M;
                P->g = g;
                P->k = reinterpret_cast<ConvKern>(k);
                r.cls = STK_MDRS;
                r.key = stkKey((const void*)k, g.x, g.z);
                r.pay = std::move(P);
            }
            issueRec(d, std::move(r));
        });
        checkLaunch(d, "conv_mdrs");
    }
    // out_i = (acc_i - NTT(y_i)) (P q_l)^-1 + d_i q_l^-1
    RowGroup B = rowsOf(2, l, sfp_limbs{l, l, 0, 0});
    B.src = B.dst = RowPtr{scr, (long long)l * n, (long long)n};
    if (md) {  // the conversion and the dropped row's lift in the forward COL pass (k_moddown_col)
        B.md = md;
        B.copy = RowPtr{acc + (size_t)ell * n, (long long)accStride, (long long)n};
        B.pre = RowPtr{acc + (size_t)l * n, (long long)accStride, (long long)n};
        B.cRows = c->ns + 1;  // (source rows per polynomial: graph byte accounting)
    }
    B.epi = 1;
    B.ein = RowPtr{acc, (long long)accStride, (long long)n};
    B.eout = RowPtr{out0, (long long)(out1 - out0), (long long)n};
    if (T) {
        B.tA0 = T[0];
        B.tA1 = T[1];
        B.tB0 = T[2];
        B.tB1 = T[3];
    } else {
        B.eadd = RowPtr{d0, (long long)(d1 - d0), (long long)n};
    }
    B.k = devConst(d, k1, l);
    B.kS = devConst(d, k1S, l);
    B.k2 = devConst(d, qlinv, l);
    B.k2S = devConst(d, k2S, l);
    nttRows(d, B, 0);
}

void sfp_moddown_rescale(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* d0,
                         const uint64_t* d1, uint64_t* acc, size_t accStride, uint32_t ell,
                         uint32_t K, uint32_t Lq, const sfp_conv* c, const uint64_t* pinv,
                         const uint64_t* pmod, const uint64_t* qlinv, uint64_t* scr, int rowDone) {
    moddownRescaleCore(d, out0, out1, d0, d1, nullptr, acc, accStride, ell, K, Lq, c, pinv, pmod, qlinv, scr,
                       rowDone);
}

int sfp_mult_relin_rescale(sfp_dev* d, uint64_t* out0, uint64_t* out1, const uint64_t* a0, const uint64_t* a1,
                           const uint64_t* b0, const uint64_t* b1, uint32_t ell, uint32_t K, uint32_t Lq,
                           uint32_t alpha, const sfp_conv* const* convs, const uint64_t* key, const sfp_conv* c,
                           const uint64_t* pinv, const uint64_t* pmod, const uint64_t* qlinv, uint64_t* acc,
                           uint64_t* ext, uint64_t* scr) {
    const uint32_t beta = (ell + alpha - 1) / alpha;
    if (!ksFuse() || d->n <= (uint32_t)kNttTile) return -1;
    if (ell < 2 || beta > (uint32_t)kMaxConvJobs || ell + K > SFP_MAX_LIMBS) {
        record(d, "mult_relin_rescale (too many digits / limbs)", hipErrorInvalidValue);
        return 0;
    }
    const uint64_t* T[4] = {a0, a1, b0, b1};
    // d2 = a1 b1 in the ModUp's first pass and the own digits; d0, d1 at row
    // ell - 1 in the inner product's fold, the rest in the ModDown's epilogue
    modupInnerCore(d, acc, acc + (size_t)(ell + K) * d->n, a1, b1, ell, K, Lq, alpha, convs, key, nullptr, nullptr,
                   T, pmod[ell - 1], 0, ell - 1, ext, scr);
    moddownRescaleCore(d, out0, out1, nullptr, nullptr, T, acc, (size_t)(ell + K) * d->n, ell, K, Lq, c, pinv, pmod,
                       qlinv, scr, 1);
    return 0;
}

// ---- sampling ----
void sfp_sample_uniform(sfp_dev* d, uint64_t* p, sfp_limbs m, uint64_t seed) {
    if (!limbsOk(d, m, "uniform")) return;
    const size_t total = (size_t)m.count * d->n;
    SFP_GO(k_uniform, dim3(ewGrid(total)), dim3(kThreads), p, m, seed, d->bar,
                       d->logn);
    checkLaunch(d, "uniform");
}

void sfp_load_i64(sfp_dev* d, uint64_t* p, const int64_t* c, sfp_limbs m) {
    if (!limbsOk(d, m, "load_i64")) return;
    // the bounce buffer is free once every lane has drained; the kernel
    // reads the coefficients straight from it
    syncAll(d);
    std::memcpy(d->bounce, c, (size_t)d->n * 8);
    SFP_GO(k_load_i64, dim3(ewGrid(d->n)), dim3(kThreads), p,
                       (const int64_t*)d->bounce, m, d->bar, d->logn);
    checkLaunch(d, "load_i64");
}



// ---- CKKS encoding on the device (the sort's in-loop masks) ----------------
// The host encoder's special inverse FFT (core/encoder.cpp fftSpecialInv),
// operation for operation: the same stage order, the same integer twiddle
// index, u = a + b and w = (a - b) * ksi with the complex product formed as
// (re re - im im, re im + im re) with no fused multiply-add, the bit
// reversal, the division by the size, then round(u * scale) and the residues
// -- so the result equals ckks_encode + sfp_load_i64 bit for bit (the host's
// doubles are IEEE-754 too, and its compiler does not contract either).
// Stages whose butterflies span more than kEncTile values run one kernel per
// stage over the whole vector; the rest run in LDS, one tile per block.
constexpr uint32_t kEncTile = 2048;  // complex values per LDS tile (32 KB)

__device__ __forceinline__ void encButterfly(double2& a, double2& b, uint32_t j, uint32_t len, const u64* rot,
                                             const double2* ksi, u64 M) {
#pragma clang fp contract(off)
    const u64 lenq = (u64)len << 2;
    const u64 idx = (lenq - (rot[j] & (lenq - 1))) * (M / lenq);  // == (lenq - rot % lenq) * M / lenq
    const double2 k = ksi[idx];
    const double2 u = make_double2(a.x + b.x, a.y + b.y);
    const double dre = a.x - b.x, dim = a.y - b.y;
    const double wre = dre * k.x - dim * k.y;
    const double wim = dre * k.y + dim * k.x;
    a = u;
    b = make_double2(wre, wim);
}

// v = the values zero-padded to S (real: imaginary parts 0)
__global__ __launch_bounds__(kThreads) void k_enc_load(double2* __restrict__ v, const double* __restrict__ vals,
                                                       uint32_t nvals, int real, uint32_t S) {
    // batch b = blockIdx.y: its own S values and nvals inputs
    v += (size_t)blockIdx.y * S;
    if (vals) vals += (size_t)blockIdx.y * nvals * (real ? 1 : 2);
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < S; i += gridDim.x * kThreads) {
        double2 x = make_double2(0.0, 0.0);
        if (i < nvals) x = real ? make_double2(vals[i], 0.0) : make_double2(vals[2 * i], vals[2 * i + 1]);
        v[i] = x;
    }
}

// one stage of butterfly span `len` over the whole vector
__global__ __launch_bounds__(kThreads) void k_enc_stage(double2* __restrict__ v, uint32_t S, uint32_t len,
                                                        const u64* __restrict__ rot,
                                                        const double2* __restrict__ ksi, u64 M) {
    v += (size_t)blockIdx.y * S;
    const uint32_t lenh = len >> 1;
    for (uint32_t t = blockIdx.x * kThreads + threadIdx.x; t < S / 2; t += gridDim.x * kThreads) {
        const uint32_t j = t % lenh, i = (t / lenh) * len;
        double2 a = v[i + j], b = v[i + j + lenh];
        encButterfly(a, b, j, len, rot, ksi, M);
        v[i + j] = a;
        v[i + j + lenh] = b;
    }
}

// the stages of span T, T/2, ..., 2 on one T-value tile per block, in LDS
__global__ __launch_bounds__(kThreads) void k_enc_tile(double2* __restrict__ v, uint32_t T,
                                                       const u64* __restrict__ rot, const double2* __restrict__ ksi,
                                                       u64 M) {
    __shared__ double2 sh[kEncTile];
    double2* g = v + (size_t)blockIdx.y * gridDim.x * T + (size_t)blockIdx.x * T;
    for (uint32_t i = threadIdx.x; i < T; i += kThreads) sh[i] = g[i];
    __syncthreads();
    for (uint32_t len = T; len >= 2; len >>= 1) {
        const uint32_t lenh = len >> 1;
        for (uint32_t t = threadIdx.x; t < T / 2; t += kThreads) {
            const uint32_t j = t % lenh, i = (t / lenh) * len;
            double2 a = sh[i + j], b = sh[i + j + lenh];
            encButterfly(a, b, j, len, rot, ksi, M);
            sh[i + j] = a;
            sh[i + j + lenh] = b;
        }
        __syncthreads();
    }
    for (uint32_t i = threadIdx.x; i < T; i += kThreads) g[i] = sh[i];
}

// coefficient x of the sparse packing (gap = n/2S): the bit-reversed value,
// divided by S, times the scale, rounded; its residue in every row of m
__global__ __launch_bounds__(kThreads) void k_enc_round(u64* __restrict__ p, const double2* __restrict__ v,
                                                        uint32_t logS, double scale, sfp_limbs m,
                                                        const sf_barrett* __restrict__ bar, uint32_t logn,
                                                        size_t pStride) {
#pragma clang fp contract(off)
    const uint32_t n = 1u << logn, half = n >> 1, gap = half >> logS;
    p += (size_t)blockIdx.y * pStride;
    v += (size_t)blockIdx.y << logS;
    for (uint32_t x = blockIdx.x * kThreads + threadIdx.x; x < n; x += gridDim.x * kThreads) {
        const uint32_t xi = x < half ? x : x - half;
        int64_t c = 0;
        if ((xi & (gap - 1)) == 0) {
            const uint32_t i = xi / gap;
            const uint32_t r = logS ? (__brev(i) >> (32 - logS)) : 0u;
            const double2 u = v[r];
            const double q = (x < half ? u.x : u.y) / (double)(1u << logS);
            c = (int64_t)rint(q * scale);
        }
        const u64 a = c < 0 ? (u64)(-(c + 1)) + 1 : (u64)c;
        for (uint32_t limb = 0; limb < m.count; ++limb) {
            const sf_barrett B = loadBar(bar, primeOf(m, limb));
            const u64 res = sf_reduce128(a, 0, &B);
            p[((size_t)limb << logn) + x] = (c < 0 && res) ? B.q - res : res;
        }
    }
}

void sfp_encode_setup(sfp_dev* d, const uint64_t* rot, const double* ksi) {
    if (!d->encRot && (hipMalloc((void**)&d->encRot, (size_t)d->n / 2 * 8) != hipSuccess ||
                       hipMalloc((void**)&d->encKsi, (size_t)(2 * d->n + 1) * sizeof(double2)) != hipSuccess)) {
        hipGetLastError();
        return record(d, "encode tables", hipErrorOutOfMemory);
    }
    hostToDev(d, d->encRot, rot, (size_t)d->n / 2 * 8);
    hostToDev(d, d->encKsi, ksi, (size_t)(2 * d->n + 1) * sizeof(double2));
}

void sfp_encode_batch(sfp_dev* d, uint64_t* dst, size_t dstStride, const double* vals, uint32_t nvals,
                      uint32_t count, int real, uint32_t slots, double scale, sfp_limbs m, uint64_t* scratch) {
    if (!count) return;
    if (!limbsOk(d, m, "encode")) return;
    if (!d->encRot || !slots || (slots & (slots - 1)) || slots > d->n / 2 || nvals > slots || count > 65535u) {
        record(d, "encode (tables not set up, or a bad slot / batch count)", hipErrorInvalidValue);
        return;
    }
    // the values travel through the argument ring: batches whose values
    // exceed half of it are encoded in chunks (ringPut refuses an upload
    // larger than the ring; a bootstrap's diagonals at 2^14+ slots are)
    const size_t per = (size_t)nvals * (real ? 8 : 16);
    const uint32_t chunk = per ? (uint32_t)std::max<size_t>(1, std::min<size_t>(count, d->ringCap / 2 / per)) : count;
    if (chunk < count && !d->capture) {
        for (uint32_t b0 = 0; b0 < count; b0 += chunk)
            sfp_encode_batch(d, dst + (size_t)b0 * dstStride, dstStride, vals + (size_t)b0 * nvals * (real ? 1 : 2),
                             nvals, std::min(chunk, count - b0), real, slots, scale, m, scratch);
        return;
    }
    const u64 M = 2ull * d->n;
    double2* v = reinterpret_cast<double2*>(scratch);
    const double* dv = nvals ? (const double*)ringPut(d, vals, (size_t)count * per) : nullptr;
    if (nvals && !dv) return;
    SFP_GO(k_enc_load, dim3(gridFor(slots, kThreads), count), dim3(kThreads), v, dv, nvals,
                       real, slots);
    const uint32_t T = std::min(slots, kEncTile);
    for (uint32_t len = slots; len > T; len >>= 1)
        SFP_GO(k_enc_stage, dim3(gridFor(slots / 2, kThreads), count), dim3(kThreads), v,
                           slots, len, d->encRot, d->encKsi, M);
    if (T >= 2)
        SFP_GO(k_enc_tile, dim3(slots / T, count), dim3(kThreads), v, T, d->encRot,
                           d->encKsi, M);
    const uint32_t logS = (uint32_t)__builtin_ctz(slots);
    SFP_GO(k_enc_round, dim3(ewGrid(d->n), count), dim3(kThreads), dst, v, logS, scale, m,
                       d->bar, d->logn, dstStride);
    checkLaunch(d, "encode");
}

void sfp_encode(sfp_dev* d, uint64_t* dst, const double* vals, uint32_t nvals, int real, uint32_t slots,
                double scale, sfp_limbs m, uint64_t* scratch) {
    sfp_encode_batch(d, dst, 0, vals, nvals, 1, real, slots, scale, m, scratch);
}

// ---- limb sharding ----
// dst row i = src row rows[i]
__global__ __launch_bounds__(kThreads) void k_gather_rows(ulonglong2* __restrict__ dst,
                                                          const ulonglong2* __restrict__ src,
                                                          const uint32_t* __restrict__ rows, uint32_t logn) {
    const uint32_t half = 1u << (logn - 1);  // 16-byte pairs per row
    const uint32_t i = blockIdx.y;
    const uint32_t r = rows[i];
    for (uint32_t x = blockIdx.x * kThreads + threadIdx.x; x < half; x += gridDim.x * kThreads)
        dst[(size_t)i * half + x] = src[(size_t)r * half + x];
}

void sfp_gather_rows(sfp_dev* d, uint64_t* dst, const uint64_t* src, const uint32_t* rows, uint32_t count) {
    if (!count) return;
    const uint32_t* dr = (const uint32_t*)ringPut(d, rows, (size_t)count * 4);
    const dim3 g(std::max(1u, std::min(64u, (d->n / 2) / kThreads)), count);
    SFP_GO(k_gather_rows, g, dim3(kThreads), (ulonglong2*)dst, (const ulonglong2*)src, dr,
                       d->logn);
    checkLaunch(d, "gather_rows");
}

void sfp_rescale_rows(sfp_dev* d, uint64_t* out, const uint64_t* in, const uint64_t* last, uint32_t dropPrime,
                      sfp_limbs m, const uint64_t* qlinv, uint32_t npoly, size_t inStride, size_t outStride,
                      size_t lastStride) {
    const uint32_t n = d->n, cnt = m.count;
    if (!cnt || !npoly) return;
    if (cnt > SFP_MAX_LIMBS || dropPrime >= d->np || !limbsOk(d, m, "rescale_rows")) {
        record(d, "rescale_rows", hipErrorInvalidValue);
        return;
    }
    u64* tmp = scratch(d, (size_t)npoly * cnt * n);
    if (!tmp) return;
    RowGroup B = rowsOf(npoly, cnt, m);
    B.src = RowPtr{last, (long long)lastStride, 0};
    B.lift = 1;
    B.liftPrime = dropPrime;
    B.dst = RowPtr{tmp, (long long)cnt * n, (long long)n};
    B.epi = 1;
    B.ein = RowPtr{in, (long long)inStride, (long long)n};
    B.eout = RowPtr{out, (long long)outStride, (long long)n};
    const u64 ql = d->hbar[dropPrime].q;
    u64 kS[SFP_MAX_LIMBS], lsub[SFP_MAX_LIMBS];
    for (uint32_t i = 0; i < cnt; ++i) {
        const u64 q = d->hbar[sfp_prime_of(m, i)].q;
        kS[i] = sf_shoup_precomp(qlinv[i], q);
        lsub[i] = ql % q;
    }
    B.k = devConst(d, qlinv, cnt);
    B.kS = devConst(d, kS, cnt);
    B.liftSub = devConst(d, lsub, cnt);
    nttRows(d, B, 0);
}

void sfp_ks_inner_map(sfp_dev* d, uint64_t* acc0, uint64_t* acc1, const uint64_t* ext, size_t extStride,
                      const uint64_t* key, uint32_t beta, sfp_limbs pm, uint32_t keyQ, uint32_t keyRows,
                      int accum) {
    if (!pm.count || !limbsOk(d, pm, "ks_inner_map")) return;
    const size_t total = (size_t)pm.count * d->n;
    timedLaunch(d, SFP_FAM_KSINNER, 8.0 * total * (3.0 * beta + (accum ? 4.0 : 2.0)), [&] {
        issueY<KsInnerArgs>(d, k_ks_inner<1>, k_ks_inner<2>, k_ks_inner<4>, dim3(ewGrid(total / 2)),
                                KsInnerArgs{acc0, acc1, ext, extStride, key, beta, pm, keyQ, keyRows, (const u64*)nullptr, (const u64*)nullptr, (u64)0, accum, (const u64*)nullptr, d->kg, 0u});
    });
    checkLaunch(d, "ks_inner_map");
}

void sfp_set_key_geom(sfp_dev* d, const sfp_key_geom* g) {
    stackFlush(d);  // (recorded launches keep the geometry they were issued with)
    d->kg = g ? *g : sfp_key_geom{};
}

int sfp_comm_uid(void* uid128) {
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
    if (!rcclApi().ok) return -1;
    return rcclApi().getUniqueId(reinterpret_cast<ncclUniqueId*>(uid128)) == ncclSuccess ? 0 : -1;
}

static void ncclCheck(sfp_dev* d, const char* what, ncclResult_t r);

static ncclComm_t rcclInit(sfp_dev* d, int rank, int world, const void* uid128) {
    ncclUniqueId id;
    std::memcpy(&id, uid128, sizeof id);
    SFP_CHECK(hipSetDevice(d->device));
    if (!rcclApi().ok) {
        std::lock_guard<std::mutex> g(d->mu);
        if (d->err.empty()) d->err = "RCCL library (librccl.so.1) not found";
        return nullptr;
    }
    ncclComm_t c = nullptr;
    const ncclResult_t r = rcclApi().commInitRank(&c, world, id, rank);
    if (r != ncclSuccess) {
        std::lock_guard<std::mutex> g(d->mu);
        if (d->err.empty()) d->err = std::string("ncclCommInitRank: ") + rcclApi().errorString(r);
        return nullptr;
    }
    return c;
}

int sfp_comm_init_rccl(sfp_dev* d, int rank, int world, const void* uid128) {
    ncclComm_t c = rcclInit(d, rank, world, uid128);
    if (!c) return -1;
    d->nccl = c;
    d->rank = rank;
    d->world = world;
    return 0;
}

int sfp_group_init_rccl(sfp_dev* d, int group, int groups, const void* uid128) {
    ncclComm_t c = rcclInit(d, group, groups, uid128);
    if (!c) return -1;
    d->gnccl = c;
    d->grank = group;
    d->gworld = groups;
    return 0;
}

void sfp_group_set_host(sfp_dev* d, int group, int groups, sfp_host_allgather_fn ag, void* user) {
    d->grank = group;
    d->gworld = groups;
    d->gHostAg = ag;
    d->gHostUser = user;
}

// One collective of sfp_comm_stats: counted, and bracketed by events on its
// stream when timing is on and nothing is being captured.
template <class F>
static void commIssue(sfp_dev* d, double received, F&& go) {
    d->commCalls++;
    d->commBytes += received;
    if (!d->commTimed || d->capture) return go();
    hipEvent_t a = takeEvent(d), b = takeEvent(d);
    SFP_CHECK(hipEventRecord(a, d->st()));
    go();
    SFP_CHECK(hipEventRecord(b, d->st()));
    d->commEv.push_back({a, b});
}

void sfp_comm_stats_reset(sfp_dev* d, int timed) {
    syncAll(d);
    for (auto& e : d->commEv) {
        d->evPool.push_back(e.first);
        d->evPool.push_back(e.second);
    }
    d->commEv.clear();
    d->commCalls = 0;
    d->commBytes = 0;
    d->commTimed = timed != 0;
}

void sfp_comm_stats(sfp_dev* d, uint64_t* calls, double* bytes, double* ms) {
    syncAll(d);
    double t = 0;
    for (auto& e : d->commEv) {
        float x = 0;
        if (hipEventElapsedTime(&x, e.first, e.second) == hipSuccess) t += x;
    }
    if (calls) *calls = d->commCalls;
    if (bytes) *bytes = d->commBytes;
    if (ms) *ms = t;
}

void sfp_group_allgather(sfp_dev* d, const void* send, void* recv, size_t bytes) {
    if (d->gnccl) {
        stackFlush(d);  // (collectives are issued in program order)
        commIssue(d, (double)bytes * (d->gworld - 1), [&] {
            ncclCheck(d, "ncclAllGather (groups)",
                      rcclApi().allGather(send, recv, bytes, ncclUint8, d->gnccl, d->st()));
        });
        return;
    }
    if (d->gworld == 1) {
        if (send != recv) sfp_d2d(d, recv, send, bytes);
        return;
    }
    if (!d->gHostAg) {
        record(d, "group allgather (no communicator)", hipErrorInvalidValue);
        return;
    }
    commIssue(d, (double)bytes * (d->gworld - 1), [&] {
        std::vector<char> hs(bytes), hr(bytes * d->gworld);
        devToHost(d, hs.data(), send, bytes);
        d->gHostAg(d->gHostUser, hs.data(), hr.data(), bytes);
        hostToDev(d, recv, hr.data(), hr.size());
    });
}

void sfp_comm_set_host(sfp_dev* d, int rank, int world, sfp_host_allgather_fn ag, sfp_host_bcast_fn bc,
                       void* user) {
    d->rank = rank;
    d->world = world;
    d->hostAg = ag;
    d->hostBc = bc;
    d->hostUser = user;
}

static void ncclCheck(sfp_dev* d, const char* what, ncclResult_t r) {
    if (r == ncclSuccess) return;
    std::lock_guard<std::mutex> g(d->mu);
    if (d->err.empty()) d->err = std::string(what) + ": " + rcclApi().errorString(r);
}

int sfp_comm_capturable(sfp_dev* d) { return (d->nccl || !d->hostAg) && (d->gnccl || !d->gHostAg) ? 1 : 0; }

void sfp_allgather(sfp_dev* d, const void* send, void* recv, size_t bytes) {
    if (d->world == 1 && !d->nccl) {
        if (send != recv) sfp_d2d(d, recv, send, bytes);
        return;
    }
    if (d->nccl) {
        stackFlush(d);  // (collectives are issued in program order)
        commIssue(d, (double)bytes * (d->world - 1), [&] {
            ncclCheck(d, "ncclAllGather", rcclApi().allGather(send, recv, bytes, ncclUint8, d->nccl, d->st()));
        });
        return;
    }
    if (!d->hostAg) {
        record(d, "allgather (no communicator)", hipErrorInvalidValue);
        return;
    }
    commIssue(d, (double)bytes * (d->world - 1), [&] {
        std::vector<char> hs(bytes), hr(bytes * d->world);
        devToHost(d, hs.data(), send, bytes);
        d->hostAg(d->hostUser, hs.data(), hr.data(), bytes);
        hostToDev(d, recv, hr.data(), hr.size());
    });
}

void sfp_bcast(sfp_dev* d, void* buf, size_t bytes, int root) {
    if (d->world == 1 && !d->nccl) return;
    const double got = d->rank == root ? 0.0 : (double)bytes;
    if (d->nccl) {
        stackFlush(d);  // (collectives are issued in program order)
        commIssue(d, got, [&] {
            ncclCheck(d, "ncclBroadcast", rcclApi().broadcast(buf, buf, bytes, ncclUint8, root, d->nccl, d->st()));
        });
        return;
    }
    if (!d->hostBc) {
        record(d, "bcast (no communicator)", hipErrorInvalidValue);
        return;
    }
    commIssue(d, got, [&] {
        std::vector<char> h(bytes);
        devToHost(d, h.data(), buf, bytes);
        d->hostBc(d->hostUser, h.data(), bytes, root);
        hostToDev(d, buf, h.data(), bytes);
    });
}
