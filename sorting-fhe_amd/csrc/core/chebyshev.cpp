// Chebyshev-series evaluation for the sinc placement and g_4 sign polynomial.
//
// Reference call sites: src/sort_algo.h:727-728 (doubled-sinc, degree 1662
// at N=256) and src/sign.cpp:76 (g_4, degree 27); both go to OpenFHE's
// EvalChebyshevSeriesPS with coefficients in the c0/2 convention
// (tests/SincTest.cpp:17-39).
//
// Algorithm (this engine's own, depth-exact):
//   baby steps  T_1..T_k, k = 2^l        (T_j at depth ceil(log2 j))
//   giant steps T_{2^i}, i = l+1..D-1    (T_{2^i} at depth i)
//   p = q * T_M + r  (Chebyshev division, M a power of two) recursively;
//   leaves sum_j a_j T_j (j <= k) are ONE fused weighted-sum kernel plus a
//   rescale.  With depth budget D this reaches degree 2^D - 2^l, which is
//   exactly OpenFHE's published depth table (≤5:3, ≤13:4, ≤27:5, ≤59:6,
//   ≤119:7, ≤247:8, ≤495:9, ≤1007:10, ≤2031:11, ≤4031:12, ≤8127:13).
//   l is chosen to minimise ciphertext products inside the budget; if the
//   evaluation lands shallower than OpenFHE's depth the result is level-
//   adjusted so the per-N multDepth tables (src/sort_algo.h:94-198) are
//   consumed exactly.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>

#include "state.h"

namespace lbcrypto {

uint32_t ChebyshevPSDepth(uint32_t d) {
    if (d <= 1) return 1;
    if (d == 2) return 2;
    static const uint32_t ub[] = {5, 13, 27, 59, 119, 247, 495, 1007, 2031, 4031, 8127, 16255, 32511, 65023};
    for (uint32_t i = 0; i < sizeof(ub) / sizeof(ub[0]); ++i)
        if (d <= ub[i]) return 3 + i;
    SFHE_THROW("Chebyshev degree too large");
}

std::vector<double> EvalChebyshevCoefficients(std::function<double(double)> func, double a,
                                              double b, uint32_t degree) {
    if (!degree) SFHE_THROW("degree must be positive");
    const double bMinusA = 0.5 * (b - a), bPlusA = 0.5 * (b + a);
    const double piByDeg = M_PI / (double)degree;
    std::vector<double> fx(degree);
    for (uint32_t j = 0; j < degree; ++j) fx[j] = func(std::cos(piByDeg * (j + 0.5)) * bMinusA + bPlusA);
    // O(degree^2) (the sinc tables interpolate at degree 13011): over the cores
    // cos(pi * i * (2j+1) / (2 d)) depends only on i*(2j+1) mod 4d
    const uint64_t P = 4ull * degree;
    std::vector<double> ctab(P);
    for (uint64_t m = 0; m < P; ++m) ctab[m] = std::cos(M_PI * (double)m / (2.0 * degree));
    std::vector<double> c(degree, 0.0);
    const double mult = 2.0 / (double)degree;
    ParallelFor(degree, [&](size_t i) {
        double acc = 0.0;
        uint64_t step = (2ull * i) % P, idx = i % P;
        for (uint32_t j = 0; j < degree; ++j) {
            acc += fx[j] * ctab[idx];
            idx += step;
            if (idx >= P) idx -= P;
        }
        c[i] = acc * mult;
    });
    return c;
}

namespace {

using Ct = Ciphertext<DCRTPoly>;

struct Val {
    bool isConst = true;
    double c = 0.0;
    Ct ct;
    int node = -1;  // PSEvaluator::build: the value of node `node` once evaluated
};

// SFHE_PS_WAVES=0: the recursive evaluation order (every product in turn)
// instead of the level-synchronous one (A/B knob; the same values)
bool psWaves() {
    static const bool on = [] {
        const char* v = std::getenv("SFHE_PS_WAVES");
        return !v || *v != '0';
    }();
    return on;
}

class PSEvaluator {
  public:
    PSEvaluator(CryptoContextImpl<DCRTPoly>* cc, const Ct& y, uint32_t l, uint32_t D)
        : cc(cc), l(l), k(1u << l), D(D) {
        T.resize(k + 1);
        T[1] = y;
        // T_2a = 2 T_a^2 - 1, T_2a+1 = 2 T_a T_a+1 - T_1, the factor 2 taken on
        // an operand: doubling the product after its rescale would double the
        // rescale's rounding error too, and at the extrema of T_a (|T_a| = 1,
        // where the error of each doubling already grows 4x) that is what
        // the series' error is made of.  (A lazily rescaled product gets the
        // same by adding before its rescale; the series holds those off.)
        // T_j for j in (2^i, 2^(i+1)] reads T_m with m <= 2^i only: each such
        // range is one wave of independent products (EvalMultMany)
        for (uint32_t half = 1; half < k; half *= 2) {
            const uint32_t lo = half + 1, hi = std::min(k, 2 * half);
            std::vector<Ct> as, bs;
            for (uint32_t j = lo; j <= hi; ++j) {
                as.push_back(doubled(j / 2));
                bs.push_back(j % 2 == 0 ? T[j / 2] : T[j / 2 + 1]);
            }
            std::vector<Ct> prods;
            if (psWaves()) {
                prods = cc->EvalMultMany(as, bs);
            } else {
                for (size_t i = 0; i < as.size(); ++i) prods.push_back(cc->EvalMult(as[i], bs[i]));
            }
            for (uint32_t j = lo; j <= hi; ++j) {
                const Ct& prod = prods[j - lo];
                T[j] = (j % 2 == 0) ? cc->EvalAdd(prod, -1.0) : cc->EvalSub(prod, atLevel(1, prod->GetLevel()));
            }
        }
        giant[l] = T[k];
    }

    // Collect the leaves eval() will visit, in visiting order (same control
    // flow, no ciphertext work), then compute them all: one multi-output
    // weighted sum + one batched rescale per leaf level.
    void precomputeLeaves(const std::vector<double>& p, uint32_t depth) {
        std::vector<std::pair<std::vector<double>, uint32_t>> leaves;  // (poly, weighted-sum level)
        plan(p, depth, 0, leaves);
        std::map<uint32_t, std::vector<size_t>> byLevel;
        for (size_t i = 0; i < leaves.size(); ++i) byLevel[leaves[i].second].push_back(i);
        pre.assign(leaves.size(), nullptr);
        for (auto& kv : byLevel) {
            const uint32_t L = kv.first;
            std::vector<uint32_t> js;  // inputs used by any leaf of this level
            for (uint32_t j = 1; j <= k; ++j)
                for (size_t i : kv.second)
                    if (j < leaves[i].first.size() && leaves[i].first[j] != 0.0) {
                        js.push_back(j);
                        break;
                    }
            std::vector<const uint64_t*> ins0, ins1;
            std::vector<double> sc;
            std::vector<DeviceBufferPtr> keep;
            for (uint32_t j : js) {
                const Ct& t = T[j];  // its first ellOf(L) rows; its scale is folded into the weights
                const uint64_t *r0, *r1;
                cc->RowsAt(t, L, &r0, &r1, keep);  // raw rows below: settled (and gathered into a replicated tail)
                ins0.push_back(r0);
                ins1.push_back(r1);
                sc.push_back(t->scale);
            }
            for (size_t b0 = 0; b0 < kv.second.size(); b0 += 64) {
                std::vector<std::vector<double>> w;
                const size_t b1 = std::min(kv.second.size(), b0 + 64);
                for (size_t t = b0; t < b1; ++t) {
                    const auto& pl = leaves[kv.second[t]].first;
                    std::vector<double> row;
                    for (uint32_t j : js) row.push_back(j < pl.size() ? pl[j] : 0.0);
                    w.push_back(std::move(row));
                }
                auto cts = cc->LinearWSumRescaleMulti(ins0, ins1, w, L, T[1]->GetSlots(), &sc);
                for (size_t t = b0; t < b1; ++t) pre[kv.second[t]] = cts[t - b0];
            }
        }
        nextLeaf = 0;
    }

    // The value of p at level `want`, or deeper where its inputs are deeper.
    // Every level alignment of the evaluation happens on the giant steps (one
    // memoised AdjustLevel per (M, level), shared by all nodes) or inside the
    // leaves: a leaf's weighted sum folds any input scale into its integer
    // weights and rescales once, so it is formed directly at the level its
    // consumer works at, for free.  A node q T_M + r is formed at
    // Lp = max(its natural product level, want): q wanted at Lp - 1, T_M
    // aligned to Lp - 1, r wanted at Lp -- no per-node rescale of a node's
    // operands or result.  want = 0: the natural level.
    //
    // Lanes (SFHE_PS_LANES, a sort phase that runs one batch per GPU): a
    // node's q and r subtrees are independent, so q goes to lane + span/2 and
    // r stays on `lane` until the span is used up; the engine orders every
    // cross-lane read after its writer.  Same operations, same values.
    Val eval(std::vector<double> p, uint32_t depth, uint32_t want = 0, int lane = 0, int span = 1) {
        trim(p);
        if (p.empty()) return Val{true, 0.0, nullptr};
        const uint32_t deg = (uint32_t)p.size() - 1;
        if (deg == 0) return Val{true, p[0], nullptr};
        if (deg <= k) return leaf(p, want);
        if (depth >= 1 && deg + (1u << l) <= (1u << (depth - 1))) return eval(p, depth - 1, want, lane, span);
        const uint32_t M = deg >= (1u << (depth - 1)) ? (1u << (depth - 1)) : (1u << (depth - 2));
        std::vector<double> q, r;
        divide(p, M, q, r);
        const uint32_t Lp = productLevel(q, depth, M, want);
        const int half = span / 2;
        if (half) cc->SetLane(lane + half);
        Val qv = eval(q, depth - 1, Lp - 1, half ? lane + half : lane, half ? half : 1);
        const Ct& TM = alignedPower(M, Lp - 1);
        Val out;
        out.isConst = false;
        if (qv.isConst)
            out.ct = cc->EvalMult(TM, qv.c);
        else
            out.ct = cc->EvalMult(qv.ct, TM);
        if (half) cc->SetLane(lane);
        Val rv = eval(r, depth, Lp, lane, half ? half : 1);
        if (std::getenv("SFHE_PS_DEBUG"))
            std::fprintf(stderr, "PSNODE deg %u M %u | q %s lvl %d | TM lvl %u | prod lvl %u | r %s lvl %d\n", deg, M,
                         qv.isConst ? "const" : "ct", qv.isConst ? -1 : (int)qv.ct->GetLevel(), TM->GetLevel(),
                         out.ct->GetLevel(), rv.isConst ? "const" : "ct", rv.isConst ? -1 : (int)rv.ct->GetLevel());
        if (rv.isConst) {
            if (rv.c != 0.0) out.ct = cc->EvalAdd(out.ct, rv.c);
        } else {
            out.ct = cc->EvalAdd(out.ct, rv.ct);
        }
        return out;
    }

    // ---- level-synchronous evaluation (the default) ----
    // build() runs eval()'s recursion -- same levels, same leaves in the same
    // visiting order -- but records each node q T_M + r instead of computing
    // it; run() then evaluates the tree in waves: every node whose q is ready
    // takes its product with the aligned giant step (the nodes of one (M, Lp)
    // as ONE EvalMultMany: their launches merged), then every node whose
    // product and r are ready takes its sum.  The same operations on the same
    // operands as eval(), so the same values; the chain of dependent products
    // shrinks from one per node (81 for the N = 256 doubled sinc) to the
    // tree's height.
    Val build(std::vector<double> p, uint32_t depth, uint32_t want = 0) {
        trim(p);
        if (p.empty()) return Val{true, 0.0, nullptr};
        const uint32_t deg = (uint32_t)p.size() - 1;
        if (deg == 0) return Val{true, p[0], nullptr};
        if (deg <= k) return leaf(p, want);
        if (depth >= 1 && deg + (1u << l) <= (1u << (depth - 1))) return build(p, depth - 1, want);
        const uint32_t M = deg >= (1u << (depth - 1)) ? (1u << (depth - 1)) : (1u << (depth - 2));
        std::vector<double> q, r;
        divide(p, M, q, r);
        const uint32_t Lp = productLevel(q, depth, M, want);
        Node nd;
        nd.q = build(q, depth - 1, Lp - 1);
        nd.r = build(r, depth, Lp);
        nd.M = M;
        nd.Lp = Lp;
        nodes.push_back(std::move(nd));
        Val v;
        v.isConst = false;
        v.node = (int)nodes.size() - 1;
        return v;
    }

    Val run(const Val& root) {
        if (root.node < 0) return root;
        auto ready = [&](const Val& v) { return v.isConst || v.node < 0 || nodes[v.node].hasOut; };
        auto value = [&](const Val& v) -> const Ct& { return v.node < 0 ? v.ct : nodes[v.node].out; };
        while (!nodes[root.node].hasOut) {
            bool progress = false;
            std::map<std::pair<uint32_t, uint32_t>, std::vector<size_t>> waves;  // (M, Lp) -> nodes
            for (size_t i = 0; i < nodes.size(); ++i)
                if (!nodes[i].hasProd && ready(nodes[i].q)) waves[{nodes[i].M, nodes[i].Lp}].push_back(i);
            for (auto& w : waves) {
                const Ct& TM = alignedPower(w.first.first, w.first.second - 1);
                std::vector<Ct> as, bs;
                std::vector<size_t> which;
                for (size_t i : w.second) {
                    Node& nd = nodes[i];
                    if (nd.q.isConst) {
                        nd.prod = cc->EvalMult(TM, nd.q.c);
                        nd.hasProd = true;
                        continue;
                    }
                    as.push_back(value(nd.q));
                    bs.push_back(TM);
                    which.push_back(i);
                }
                auto prods = cc->EvalMultMany(as, bs);
                for (size_t t = 0; t < which.size(); ++t) {
                    nodes[which[t]].prod = prods[t];
                    nodes[which[t]].hasProd = true;
                }
                progress = true;
            }
            // the ready sums, as batches of independent ops
            std::vector<Node*> sums;
            for (auto& nd : nodes)
                if (!nd.hasOut && nd.hasProd && ready(nd.r)) sums.push_back(&nd);
            for (size_t b0 = 0; b0 < sums.size(); b0 += batchWidth()) {
                const size_t b1 = std::min(sums.size(), b0 + batchWidth());
                BatchScope bs(cc, (uint32_t)(b1 - b0));
                for (size_t t = b0; t < b1; ++t) {
                    Node& nd = *sums[t];
                    bs.lane((uint32_t)(t - b0));
                    if (nd.r.isConst)
                        nd.out = nd.r.c != 0.0 ? cc->EvalAdd(nd.prod, nd.r.c) : nd.prod;
                    else
                        nd.out = cc->EvalAdd(nd.prod, value(nd.r));
                    nd.hasOut = true;
                    nd.prod = nullptr;
                }
                progress = true;
            }
            if (!progress) SFHE_THROW("internal: Chebyshev wave evaluation stalled");
        }
        Val out;
        out.isConst = false;
        out.ct = nodes[root.node].out;
        nodes.clear();
        return out;
    }

  private:
    struct Node {
        Val q, r;
        uint32_t M = 0, Lp = 0;
        Ct prod, out;
        bool hasProd = false, hasOut = false;
    };
    std::vector<Node> nodes;

    // p = q T_M + r (Chebyshev division by T_M, M >= deg / 2)
    static void divide(const std::vector<double>& p, uint32_t M, std::vector<double>& q, std::vector<double>& r) {
        const uint32_t deg = (uint32_t)p.size() - 1;
        q.assign(deg - M + 1, 0.0);
        r.assign(p.begin(), p.begin() + M);
        for (uint32_t j = M; j <= deg; ++j) {
            if (j == M) {
                q[0] += p[j];
            } else {
                q[j - M] += 2.0 * p[j];
                r[2 * M - j] -= p[j];
            }
        }
    }

    // eval()'s control flow without ciphertext work: the leaf polynomials with
    // the level of their weighted sum, in eval()'s visiting order.
    void plan(std::vector<double> p, uint32_t depth, uint32_t want,
              std::vector<std::pair<std::vector<double>, uint32_t>>& leaves) {
        trim(p);
        if (p.size() <= 1) return;
        const uint32_t deg = (uint32_t)p.size() - 1;
        if (deg <= k) {
            const int lv = leafSumLevel(p, want);
            if (lv >= 0) leaves.emplace_back(p, (uint32_t)lv);
            return;
        }
        if (depth >= 1 && deg + (1u << l) <= (1u << (depth - 1))) return plan(p, depth - 1, want, leaves);
        const uint32_t M = deg >= (1u << (depth - 1)) ? (1u << (depth - 1)) : (1u << (depth - 2));
        std::vector<double> q, r;
        divide(p, M, q, r);
        const uint32_t Lp = productLevel(q, depth, M, want);
        plan(q, depth - 1, Lp - 1, leaves);
        plan(r, depth, Lp, leaves);
    }

    // level of a node's product q T_M: the natural one (q and T_M as they come,
    // +1) or `want`, whichever is deeper
    uint32_t productLevel(const std::vector<double>& q, uint32_t depth, uint32_t M, uint32_t want) const {
        if (naturalOnly()) want = 0;
        const int nq = natural(q, depth - 1);
        const uint32_t nat = (uint32_t)std::max(nq, (int)powerLevel(M)) + 1;
        return std::max(nat, want);
    }

    // level eval(p, depth) reaches without a wanted level (-1: a constant)
    int natural(std::vector<double> p, uint32_t depth) const {
        trim(p);
        if (p.size() <= 1) return -1;
        const uint32_t deg = (uint32_t)p.size() - 1;
        if (deg <= k) {
            const int lv = leafSumLevel(p, 0);
            return lv < 0 ? -1 : lv + 1;
        }
        if (depth >= 1 && deg + (1u << l) <= (1u << (depth - 1))) return natural(p, depth - 1);
        const uint32_t M = deg >= (1u << (depth - 1)) ? (1u << (depth - 1)) : (1u << (depth - 2));
        std::vector<double> q, r;
        divide(p, M, q, r);
        const int lp = (int)productLevel(q, depth, M, 0);
        return std::max(lp, natural(r, depth));
    }

    // level of the leaf's weighted sum (its output is one level deeper): the
    // deepest input's, or want - 1 when that is deeper; -1 if p is a constant
    int leafSumLevel(const std::vector<double>& p, uint32_t want) const {
        if (naturalOnly()) want = 0;
        int lev = -1;
        for (uint32_t j = 1; j < p.size(); ++j)
            if (p[j] != 0.0) lev = std::max(lev, (int)T[j]->GetLevel());
        if (lev < 0) return -1;
        return std::max(lev, (int)want - 1);
    }

    // SFHE_PS_NATURAL=1: every node and leaf at its natural level, the sums
    // aligning the shallower operand (the pre-targeting plan; noise probe)
    static bool naturalOnly() {
        static const bool on = [] {
            const char* v = std::getenv("SFHE_PS_NATURAL");
            return v && *v == '1';
        }();
        return on;
    }

    static void trim(std::vector<double>& p) {
        while (!p.empty() && p.back() == 0.0) p.pop_back();
    }

    // level of T_M for a power of two M (built or not yet built)
    uint32_t powerLevel(uint32_t M) const {
        if (M <= k) return T[M]->GetLevel();
        return powerLevel(M / 2) + 1;  // T_2M = 2 T_M^2 - 1: one product
    }

    // T_M for a power of two M (giant steps built lazily: T_2M = 2 T_M^2 - 1)
    const Ct& power(uint32_t M) {
        if (M <= k) return T[M];
        uint32_t i = (uint32_t)__builtin_ctz(M);
        auto it = giant.find(i);
        if (it != giant.end()) return it->second;
        const Ct& half = power(M / 2);
        const Ct twice = cc->EvalAdd(half, half);  // 2 T_M before the rescale, as above
        return giant[i] = cc->EvalAdd(cc->EvalMult(twice, half), -1.0);
    }

    // 2 T_j, memoised (an odd T_j+1's product reuses T_j's)
    const Ct& doubled(uint32_t j) {
        auto it = twice.find(j);
        if (it != twice.end()) return it->second;
        return twice[j] = cc->EvalAdd(T[j], T[j]);
    }

    // T_M at `level` (>= its own): one AdjustLevel per (M, level), memoised
    const Ct& alignedPower(uint32_t M, uint32_t level) {
        const Ct& t = power(M);
        if (t->GetLevel() >= level) return t;
        auto key = std::make_pair(M, level);
        auto it = alignedPow.find(key);
        if (it != alignedPow.end()) return it->second;
        return alignedPow[key] = cc->AdjustLevel(t, level);
    }

    const Ct& atLevel(uint32_t j, uint32_t level) {
        auto key = std::make_pair(j, level);
        auto it = aligned.find(key);
        if (it != aligned.end()) return it->second;
        return aligned[key] = (T[j]->GetLevel() == level ? T[j] : cc->AdjustLevel(T[j], level));
    }

    Val leaf(const std::vector<double>& p, uint32_t want) {
        if (!pre.empty()) {  // precomputed (same visiting order as plan())
            bool any = false;
            for (uint32_t j = 1; j < p.size(); ++j) any = any || p[j] != 0.0;
            if (!any) return Val{true, p[0], nullptr};
            if (nextLeaf >= pre.size()) SFHE_THROW("internal: Chebyshev leaf plan mismatch");
            Val out;
            out.isConst = false;
            out.ct = pre[nextLeaf];
            pre[nextLeaf++] = nullptr;
            if (p[0] != 0.0) out.ct = cc->EvalAdd(out.ct, p[0]);
            return out;
        }
        const int lv = leafSumLevel(p, want);
        if (lv < 0) return Val{true, p[0], nullptr};
        std::vector<const uint64_t*> ins0, ins1;
        std::vector<double> w, sc;
        std::vector<DeviceBufferPtr> keep;
        for (uint32_t j = 1; j < p.size(); ++j) {
            if (p[j] == 0.0) continue;
            const Ct& t = T[j];  // unadjusted: its scale is folded into the weight
            const uint64_t *r0, *r1;
            cc->RowsAt(t, (uint32_t)lv, &r0, &r1, keep);  // raw pointers below: canonical rows, ordered after their writers
            ins0.push_back(r0);
            ins1.push_back(r1);
            w.push_back(p[j]);
            sc.push_back(t->scale);
        }
        Val out;
        out.isConst = false;
        out.ct = cc->LinearWSumRescale(ins0, ins1, w, (uint32_t)lv, T[1]->GetSlots(), &sc);
        if (p[0] != 0.0) out.ct = cc->EvalAdd(out.ct, p[0]);
        return out;
    }

    CryptoContextImpl<DCRTPoly>* cc;
    uint32_t l, k, D;
    std::vector<Ct> pre;  // precomputed leaves in visiting order
    size_t nextLeaf = 0;
    std::vector<Ct> T;
    std::map<uint32_t, Ct> giant;
    std::map<std::pair<uint32_t, uint32_t>, Ct> aligned, alignedPow;
    std::map<uint32_t, Ct> twice;
};

}  // namespace

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalChebyshevSeriesPS(
    const Ciphertext<DCRTPoly>& x, const std::vector<double>& coeffs, double a, double b) {
    OpLock g(st.get());
    // Lazy rescaling is held off inside the series: a deferred relinearisation
    // consumed by a node's sum (q T_M + r) key-switches its unrescaled rows
    // and rescales separately, where the canonical path fuses the ModDown
    // with the rescale.  Measured on the metric sort (N=256 @ 2^16): 56.4 ms
    // with lazy products in the series, 54.6 ms without, sort error 2.6e-5 vs
    // 3.2e-5.  SFHE_LAZY_PS=1 keeps them.
    static const bool lazyPs = [] {
        const char* v = std::getenv("SFHE_LAZY_PS");
        return v && *v == '1';
    }();
    struct Hold {
        SfheContextState* s;
        bool on;
        ~Hold() {
            if (on) --s->lazyHold;
        }
    } hold{st.get(), !lazyPs};
    if (hold.on) ++st->lazyHold;
    std::vector<double> p(coeffs);
    while (!p.empty() && p.back() == 0.0) p.pop_back();
    if (p.empty()) SFHE_THROW("empty Chebyshev series");
    p[0] *= 0.5;  // c0/2 convention -> true constant term
    Ciphertext<DCRTPoly> y = x;
    if (a != -1.0 || b != 1.0) {
        y = EvalMult(x, 2.0 / (b - a));
        y = EvalAdd(y, -(a + b) / (b - a));
    }
    const uint32_t d = (uint32_t)p.size() - 1;
    if (d == 0) return EvalAdd(EvalMult(y, 0.0), p[0]);
    const uint32_t D = ChebyshevPSDepth(d);
    // choose the baby-step exponent l: reach degree d within depth D with the
    // fewest ciphertext products (k-1 baby, D-1-l giant, ~d/k recursion nodes)
    uint32_t bestL = 1;
    double bestCost = 1e300;
    for (uint32_t l = 1; l + 1 <= D && l <= 6; ++l) {
        if ((1ull << D) - (1ull << l) < d) continue;
        double cost = (double)((1u << l) - 1) + (double)(D - 1 - l) + std::ceil((double)d / (1u << l));
        if (cost < bestCost) {
            bestCost = cost;
            bestL = l;
        }
    }
    static const uint32_t forceL = [] {  // SFHE_PS_L=l: the baby-step exponent for series of degree >= 64 (A/B)
        const char* v = std::getenv("SFHE_PS_L");
        return v ? (uint32_t)std::atoi(v) : 0u;
    }();
    if (forceL && d >= 64 && (1ull << D) - (1ull << forceL) >= d && forceL + 1 <= D) bestL = forceL;
    const uint32_t l = std::min(bestL, (uint32_t)(31 - __builtin_clz(std::max<uint32_t>(d, 2))));
    Ciphertext<DCRTPoly> out;
    {
        // SFHE_PS_LANES=k: the recursion's independent subtrees on k lanes,
        // when no lane region is open (a sort phase with one batch per GPU:
        // config 3, or a batch-split rank) and the context is not limb-sharded
        static const int psLanes = [] {
            const char* v = std::getenv("SFHE_PS_LANES");
            return v ? std::atoi(v) : 0;
        }();
        int lanes = 1;
        if (psLanes > 1 && !st->forkedLanes && d >= 64) {
            lanes = std::min(psLanes, LaneCount());
            lanes = lanes >= 4 ? 4 : (lanes >= 2 ? 2 : 1);
        }
        // the lane region is closed on every exit, an exception included
        struct LaneRegion {
            CryptoContextImpl<DCRTPoly>* cc;
            int lanes;
            LaneRegion(CryptoContextImpl<DCRTPoly>* c, int k) : cc(c), lanes(k) {
                if (lanes > 1) cc->ForkLanes(lanes);
            }
            ~LaneRegion() {
                if (lanes > 1) {
                    cc->SetLane(0);
                    cc->JoinLanes();
                }
            }
        } region(this, lanes);
        PSEvaluator ps(this, y, l, D);
        static const bool batched = std::getenv("SFHE_PS_UNBATCHED") == nullptr;
        if (batched) ps.precomputeLeaves(p, D);
        auto v = (lanes == 1 && psWaves()) ? ps.run(ps.build(p, D)) : ps.eval(p, D, 0, 0, lanes);
        out = v.isConst ? EvalAdd(EvalMult(y, 0.0), v.c) : v.ct;
    }
    const uint32_t target = y->GetLevel() + D;
    if (out->GetLevel() > target)
        SFHE_THROW("internal: Chebyshev evaluation exceeded OpenFHE depth");
    if (out->GetLevel() < target) out = AdjustLevel(out, target);
    return out;
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalChebyshevFunction(
    std::function<double(double)> f, const Ciphertext<DCRTPoly>& x, double a, double b,
    uint32_t degree) {
    auto c = EvalChebyshevCoefficients(f, a, b, degree + 1);
    return EvalChebyshevSeriesPS(x, c, a, b);
}

Ciphertext<DCRTPoly> CryptoContextImpl<DCRTPoly>::EvalPolyLinear(
    const Ciphertext<DCRTPoly>& x, const std::vector<double>& coeffs) {
    OpLock g(st.get());
    std::vector<double> p(coeffs);
    while (!p.empty() && p.back() == 0.0) p.pop_back();
    if (p.size() < 2) SFHE_THROW("EvalPolyLinear needs degree >= 1");
    const uint32_t d = (uint32_t)p.size() - 1;
    // only the powers the polynomial uses, and the ones they are built from
    // (x^j = x^(j/2) x^(j - j/2)): an odd polynomial skips x^6 at degree 7
    std::vector<char> need(d + 1, 0);
    for (uint32_t j = d; j >= 1; --j)
        if (p[j] != 0.0 || need[j]) {
            need[j] = 1;
            if (j >= 2) need[j / 2] = need[j - j / 2] = 1;
        }
    std::vector<Ciphertext<DCRTPoly>> pw(d + 1);
    pw[1] = x;
    // x^j for j in (2^i, 2^(i+1)] reads powers <= 2^i only: one wave of
    // independent products each (EvalMultMany; the same values)
    for (uint32_t half = 1; half < d; half *= 2) {
        std::vector<Ciphertext<DCRTPoly>> as, bs;
        std::vector<uint32_t> js;
        for (uint32_t j = half + 1; j <= std::min(d, 2 * half); ++j)
            if (need[j]) {
                as.push_back(pw[j / 2]);
                bs.push_back(pw[j - j / 2]);
                js.push_back(j);
            }
        if (psWaves()) {
            auto prods = EvalMultMany(as, bs);
            for (size_t t = 0; t < js.size(); ++t) pw[js[t]] = prods[t];
        } else {
            for (size_t t = 0; t < js.size(); ++t) pw[js[t]] = EvalMult(as[t], bs[t]);
        }
    }
    uint32_t lev = 0;
    for (uint32_t j = 1; j <= d; ++j)
        if (p[j] != 0.0) lev = std::max(lev, pw[j]->GetLevel());
    // powers below the top level enter with their own scale folded into the
    // weight (no level adjustment, no extra rounding)
    std::vector<const uint64_t*> i0, i1;
    std::vector<double> w, sc;
    std::vector<DeviceBufferPtr> keep;
    for (uint32_t j = 1; j <= d; ++j) {
        if (p[j] == 0.0) continue;
        const uint64_t *r0, *r1;
        RowsAt(pw[j], lev, &r0, &r1, keep);  // raw rows below
        i0.push_back(r0);
        i1.push_back(r1);
        w.push_back(p[j]);
        sc.push_back(pw[j]->scale);
    }
    auto out = LinearWSumRescale(i0, i1, w, lev, x->GetSlots(), &sc);
    if (p[0] != 0.0) out = EvalAdd(out, p[0]);
    return out;
}

}  // namespace lbcrypto
