// Client side of the serialized sort flow (test infrastructure): the key
// holder's half that the reference leaves to FHERMA -- generate the context
// and keys, encrypt an input array, serialize everything for src/main.cpp;
// afterwards decrypt its output and check it is the sorted input.
//   fherma_client keygen <dir> <logn> <depth> <batch> <N> <seed>
//   fherma_client check  <dir> <N> [tol]     (exit 0: max error < tol, default 0.01)
// Mirrors the reference's src/config.json parameters (ring, depth, scale 40,
// batch, rotation indexes).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "ciphertext-ser.h"
#include "cryptocontext-ser.h"
#include "key/key-ser.h"
#include "openfhe.h"

using namespace lbcrypto;

static const std::vector<int> kRot = {-1, -2, -4, -8, -16, -32, 1, 2, 4, 8, 16,
                                      32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384};

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const std::string mode = argv[1], dir = argv[2];
    if (mode == "keygen" && argc >= 8) {
        CCParams<CryptoContextCKKSRNS> p;
        p.SetRingDim(1u << std::atoi(argv[3]));
        p.SetMultiplicativeDepth(std::atoi(argv[4]));
        p.SetScalingModSize(40);
        p.SetBatchSize(std::atoi(argv[5]));
        p.SetSecurityLevel(HEStd_NotSet);
        auto cc = GenCryptoContext(p);
        cc->Enable(PKE);
        cc->Enable(KEYSWITCH);
        cc->Enable(LEVELEDSHE);
        cc->Enable(ADVANCEDSHE);
        auto kp = cc->KeyGen();
        cc->EvalMultKeyGen(kp.secretKey);
        cc->EvalRotateKeyGen(kp.secretKey, kRot);
        const int N = std::atoi(argv[6]);
        std::mt19937 rng(std::atoi(argv[7]));
        std::vector<int> perm(N);
        for (int i = 0; i < N; ++i) perm[i] = i;
        std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<double> x(N);
        for (int i = 0; i < N; ++i) x[i] = (double)perm[i] / N;
        auto ct = cc->Encrypt(kp.publicKey, cc->MakeCKKSPackedPlaintext(x));
        bool ok = Serial::SerializeToFile(dir + "/cc.bin", cc, SerType::BINARY) &&
                  Serial::SerializeToFile(dir + "/pub.bin", kp.publicKey, SerType::BINARY) &&
                  Serial::SerializeToFile(dir + "/sk.bin", kp.secretKey, SerType::BINARY) &&
                  Serial::SerializeToFile(dir + "/input.bin", ct, SerType::BINARY);
        std::ofstream mk(dir + "/mult.bin", std::ios::binary), rk(dir + "/rot.bin", std::ios::binary);
        ok = ok && CryptoContextImpl<DCRTPoly>::SerializeEvalMultKey(mk, SerType::BINARY) &&
             CryptoContextImpl<DCRTPoly>::SerializeEvalAutomorphismKey(rk, SerType::BINARY);
        std::ofstream plain(dir + "/input.txt");
        for (double v : x) plain << v << "\n";
        std::printf("keygen %s\n", ok ? "ok" : "FAILED");
        return ok ? 0 : 1;
    }
    if (mode == "check" && argc >= 4) {
        const int N = std::atoi(argv[3]);
        CryptoContext<DCRTPoly> cc;
        PrivateKey<DCRTPoly> sk;
        Ciphertext<DCRTPoly> out;
        if (!Serial::DeserializeFromFile(dir + "/cc.bin", cc, SerType::BINARY) ||
            !Serial::DeserializeFromFile(dir + "/sk.bin", sk, SerType::BINARY) ||
            !Serial::DeserializeFromFile(dir + "/output.bin", out, SerType::BINARY)) {
            std::printf("check: deserialization FAILED\n");
            return 1;
        }
        std::vector<double> x;
        std::ifstream plain(dir + "/input.txt");
        for (double v; plain >> v;) x.push_back(v);
        std::sort(x.begin(), x.end());
        Plaintext pt;
        cc->Decrypt(sk, out, &pt);
        const auto& got = pt->GetRealPackedValue();
        double err = 0;
        for (int i = 0; i < N; ++i) err = std::max(err, std::fabs(got[i] - x[i]));
        std::printf("check: level %u, max error %.3g\n", out->GetLevel(), err);
        const double tol = argc > 4 ? std::atof(argv[4]) : 0.01;
        return err < tol ? 0 : 1;
    }
    return 2;
}
