// A caller of the lbcrypto facade (tests/test_abi_stamp.py): built once as is
// and once with -DSFHE_LAYOUT_SALT=1, a stand-in for a program compiled
// against headers whose object layouts differ from the library's.
#include <cstdio>

#include "openfhe.h"

using namespace lbcrypto;

int main() {
    CCParams<CryptoContextCKKSRNS> p;
    p.SetMultiplicativeDepth(2);
    p.SetScalingModSize(40);
    p.SetRingDim(1 << 12);
    p.SetBatchSize(8);
    p.SetSecurityLevel(HEStd_NotSet);
    try {
        auto cc = GenCryptoContext(p);
        std::printf("context ring %u\n", cc->GetRingDimension());
        return 0;
    } catch (const OpenFHEException& e) {
        std::printf("OpenFHEException: %s\n", e.what());
        return 3;
    }
}
