// Reference-side driver (test infrastructure): dumps the REFERENCE's
// Decomposer<N>::decompose (src/rotation.h:30-190, compiled where it lies under
// /root/reference by oracle/Makefile's `ref` target into oracle/_ref/) for a
// range of rotations, so tests/test_decompose_ref.py can pin the engine's
// Decomposer step for step.  The reference header is named by REF_ROTATION_H;
// its own includes (openfhe.h, encryption.h, ...) resolve to the engine's
// facade headers.
//   decompose_dump N algo wrapN rmin rmax key...   (algo 0 NAF, 1 BNAF, 2 BINARY)
// prints one line per rotation: "r value:step value:step ..."
#include <cstdio>
#include <cstdlib>
#include <vector>

#include REF_ROTATION_H

template <int N>
static int dumpN(int algo, int wrapN, int rmin, int rmax, const std::vector<int>& keys) {
    Decomposer<N> d(keys);
    const DecomposeAlgo a = algo == 0 ? DecomposeAlgo::NAF : algo == 1 ? DecomposeAlgo::BNAF : DecomposeAlgo::BINARY;
    for (int r = rmin; r <= rmax; ++r) {
        std::printf("%d", r);
        for (const auto& s : d.decompose(r, wrapN, a)) std::printf(" %d:%d", (int)s.value, s.stepSize);
        std::printf("\n");
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 7) return 2;
    const int N = std::atoi(argv[1]), algo = std::atoi(argv[2]), wrapN = std::atoi(argv[3]);
    const int rmin = std::atoi(argv[4]), rmax = std::atoi(argv[5]);
    std::vector<int> keys;
    for (int i = 6; i < argc; ++i) keys.push_back(std::atoi(argv[i]));
    switch (N) {
        case 4: return dumpN<4>(algo, wrapN, rmin, rmax, keys);
        case 8: return dumpN<8>(algo, wrapN, rmin, rmax, keys);
        case 16: return dumpN<16>(algo, wrapN, rmin, rmax, keys);
        case 32: return dumpN<32>(algo, wrapN, rmin, rmax, keys);
        case 64: return dumpN<64>(algo, wrapN, rmin, rmax, keys);
        case 128: return dumpN<128>(algo, wrapN, rmin, rmax, keys);
        case 256: return dumpN<256>(algo, wrapN, rmin, rmax, keys);
        case 512: return dumpN<512>(algo, wrapN, rmin, rmax, keys);
        case 1024: return dumpN<1024>(algo, wrapN, rmin, rmax, keys);
    }
    return 2;
}
