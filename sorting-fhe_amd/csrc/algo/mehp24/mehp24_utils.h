// Helpers sort_algo.h takes from the MEHP24 utilities (reference
// src/mehp24/mehp24_utils.h:21-25, :143-155).  The MEHP24 competitor sort
// itself is out of scope; only what DirectSort's hybrid
// placement (sort_hybrid1) calls is provided.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "openfhe.h"

#define MIN(a, b) ((a) < (b) ? (a) : (b))
#define MAX(a, b) ((a) > (b) ? (a) : (b))
#define MIN_VEC(V) *std::min_element(V.begin(), V.end())
#define MAX_VEC(V) *std::max_element(V.begin(), V.end())
#define LOG2(X) (size_t) std::ceil(std::log2((X)))

namespace mehp24 {
namespace utils {

// Step function (sign(x) + 1) / 2 on [-1, 1]: dg applications of the
// degree-7 g3, df - 1 of f3 and a final f3 / 2 + 1/2, each one
// EvalPolyLinear (4 levels) -- reference mehp24_utils.cpp:246-261.
lbcrypto::Ciphertext<lbcrypto::DCRTPoly> signAdv(lbcrypto::Ciphertext<lbcrypto::DCRTPoly>& c, const size_t dg,
                                                 const size_t df);

// ~1 where the slot holds 0, ~0 at every other integer in (-b, b):
// step(x/b + 1/(2b)) * (1 - step(x/b - 1/(2b))) -- reference :166-174.
// Levels: 1 (x 1/b) + 4 (dg + df) (signAdv) + 1 (product).
lbcrypto::Ciphertext<lbcrypto::DCRTPoly> indicatorAdv(const lbcrypto::Ciphertext<lbcrypto::DCRTPoly>& c,
                                                      const double b, const size_t dg, const size_t df);

// Polynomial degree that fits a multiplicative depth (reference :215-244).
uint32_t depth2degree(const uint32_t depth);

// Rotation amounts of the MEHP24 matrix helpers (reference :182-213).
std::vector<int32_t> getRotationIndices(const size_t matrixSize);

}  // namespace utils
}  // namespace mehp24
