// Dependent-chain latency of the evaluator's ops (developer tool): a chain of
// R dependent ops is captured into one hipGraph and replayed -- the sort's
// steady state, where a product waits for the one before it -- and reported
// per op.  Links the product library:
//   make -C tools chainbench && tools/build/chainbench [reps]
// Chains (ring 2^16, depth 34, scale 40 -- the metric sort's context):
//   mult  ell0..   x <- x * x (canonical: relinearised and rescaled), ell0 down
//   mult2 ell0..   two independent chains as one batched op per step
//   lanes ell0..   two independent chains on two lanes (the sort's batches)
//   rsc   ell      x <- Rescale(x * c) at a fixed limb count
//   rot   ell      x <- Rotate(x, 1) at a fixed limb count
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "openfhe.h"
#include "prims.h"
#include "state.h"
#include "rotation.h"

using namespace lbcrypto;

using Ct = Ciphertext<DCRTPoly>;

static CryptoContext<DCRTPoly> cc;

// (SFHE_NTT_TRACE builds of the library: k_mdrsf's per-phase clocks)
extern "C" int sfp_mdrs_trace(sfp_dev* d, unsigned long long* out8);
static void mdrsTrace(bool print) {
    unsigned long long t[8];
    if (sfp_mdrs_trace(cc->state()->dev, t) != 0 || !print || !t[7]) return;
    std::printf("       k_mdrsf blocks=%llu clk/block: load+constants %6.0f  y %6.0f  overflow+r %6.0f  phase2+store %6.0f\n",
                t[7], (double)t[0] / t[7], (double)t[1] / t[7], (double)t[2] / t[7], (double)t[3] / t[7]);
}

static Ct atEll(const Ct& x, uint32_t ell) {
    Ct y = x->Clone();
    const uint32_t lq = cc->state()->Lq;
    cc->LevelReduceInPlace(y, nullptr, lq - ell - y->GetLevel());
    cc->Settle(y);
    return y;
}

// capture body(in) -> out, replay `reps` times; microseconds per replay
template <class F>
static double chain(const Ct& in, int reps, F&& body, size_t* nodes) {
    Ct warm = body(in);  // eager pass (builds tables / plaintexts)
    cc->Settle(warm);
    cc->Synchronize();
    if (!cc->BeginCapture()) return -1.0;
    Ct out = body(in);
    cc->Settle(out);
    auto g = cc->EndCapture(out);
    if (!g) return -1.0;
    *nodes = cc->GraphNodes(g);
    cc->Launch(g);
    cc->Synchronize();
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < reps; ++i) cc->Launch(g);
    cc->Synchronize();
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    // argv[2]: which chains ("all", or a comma list of mult,mult2,lanes,rot,rsc)
    const std::string only = argc > 2 ? argv[2] : "all";
    auto want = [&](const char* c) { return only == "all" || ("," + only + ",").find("," + std::string(c) + ",") != std::string::npos; };
    const int R = 8;
    CCParams<CryptoContextCKKSRNS> p;
    p.SetMultiplicativeDepth(34);
    p.SetScalingModSize(40);
    p.SetRingDim(1u << 16);
    p.SetBatchSize(256);
    p.SetSecurityLevel(HEStd_NotSet);
    cc = GenCryptoContext(p);
    cc->Enable(PKE);
    cc->Enable(KEYSWITCH);
    cc->Enable(LEVELEDSHE);
    auto kp = cc->KeyGen();
    cc->EvalMultKeyGen(kp.secretKey);
    std::vector<int> baby;
    for (int k = 1; k < 16; ++k) baby.push_back(k);
    cc->EvalRotateKeyGen(kp.secretKey, baby);
    std::vector<double> v(256);
    for (int i = 0; i < 256; ++i) v[i] = 0.5 + 0.001 * i;
    Ct x0 = cc->Encrypt(kp.publicKey, cc->MakeCKKSPackedPlaintext(v));
    setvbuf(stdout, nullptr, _IONBF, 0);
    std::printf("%-6s %5s %4s %8s %10s %10s\n", "chain", "ell", "ops", "nodes", "us/replay", "us/op");
    auto report = [&](const char* name, uint32_t ell, int ops, double us, size_t nodes) {
        std::printf("%-6s %5u %4d %8zu %10.1f %10.2f\n", name, ell, ops, nodes, us, us / ops);
    };
    for (uint32_t ell0 : {10u, 13u, 20u, 35u}) {
        Ct x = atEll(x0, ell0);
        size_t nodes = 0;
        double us = 0;
        if (want("mult")) {
            mdrsTrace(false);
            us = chain(x, reps, [&](const Ct& in) {
                Ct y = in;
                for (int k = 0; k < R; ++k) y = cc->EvalMultMany({y}, {y})[0];
                return y;
            }, &nodes);
            report("mult", ell0, R, us, nodes);
            mdrsTrace(true);
        }
        if (want("mult2")) {
        us = chain(x, reps, [&](const Ct& in) {
            Ct y = in, z = cc->EvalAdd(in, 0.25);
            cc->Settle(z);
            for (int k = 0; k < R; ++k) {
                auto r = cc->EvalMultMany({y, z}, {y, z});
                y = r[0];
                z = r[1];
            }
            return cc->EvalAdd(y, z);
        }, &nodes);
        report("mult2", ell0, R, us, nodes);
        }
        if (want("lanes")) {
        us = chain(x, reps, [&](const Ct& in) {
            Ct z = cc->EvalAdd(in, 0.25);
            cc->Settle(z);
            Ct a = in, b = z;
            cc->ForkLanes(2);
            cc->SetLane(0);
            for (int k = 0; k < R; ++k) a = cc->EvalMultMany({a}, {a})[0];
            cc->SetLane(1);
            for (int k = 0; k < R; ++k) b = cc->EvalMultMany({b}, {b})[0];
            cc->SetLane(0);
            cc->JoinLanes();
            return cc->EvalAdd(a, b);
        }, &nodes);
        report("lanes", ell0, R, us, nodes);
        }
    }
    // hoist: the rank phase's baby rotations -- 16 rotations of one ciphertext
    // sharing one ModUp (RotationComposer::rotateMany), summed
    if (want("hoist")) {
        RotationComposer<256> rot(cc, nullptr, baby);
        std::vector<int> amounts;
        for (int k = 0; k < 16; ++k) amounts.push_back(k);
        for (uint32_t ell : {35u, 20u, 13u}) {
            Ct x = atEll(x0, ell);
            size_t nodes = 0;
            const double us = chain(x, reps, [&](const Ct& in) {
                auto r = rot.rotateMany(in, amounts);
                Ct sum = r[0];
                for (size_t k = 1; k < r.size(); ++k) sum = cc->EvalAdd(sum, r[k]);
                cc->Settle(sum);
                return sum;
            }, &nodes);
            report("hoist", ell, 16, us, nodes);
        }
    }
    for (uint32_t ell : {4u, 9u, 13u, 20u, 35u}) {
        Ct x = atEll(x0, ell);
        size_t nodes = 0;
        double us = 0;
        if (want("rot")) {
        us = chain(x, reps, [&](const Ct& in) {
            Ct y = in;
            for (int k = 0; k < R; ++k) {
                y = cc->EvalRotate(y, 1);
                cc->Settle(y);
            }
            return y;
        }, &nodes);
        report("rot", ell, R, us, nodes);
        }
        if (!want("rsc") || ell + R > cc->state()->Lq) continue;
        Ct xs = atEll(x0, ell + R);
        us = chain(xs, reps, [&](const Ct& in) {
            Ct y = in;
            for (int k = 0; k < R; ++k) {
                y = cc->EvalMult(y, 1.0009765625);
                cc->Settle(y);
            }
            return y;
        }, &nodes);
        report("rsc", ell + R, R, us, nodes);
    }
    const char* e = sfp_last_error(cc->state()->dev);
    if (e) std::printf("ERROR: %s\n", e);
    return e ? 1 : 0;
}
