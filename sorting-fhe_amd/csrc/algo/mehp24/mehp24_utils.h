// Helpers sort_algo.h takes from the MEHP24 utilities (reference
// src/mehp24/mehp24_utils.h:21-25).  The MEHP24 competitor sort itself is
// out of scope.
#pragma once

#include <algorithm>
#include <cmath>

#include "openfhe.h"

#define MIN(a, b) ((a) < (b) ? (a) : (b))
#define MAX(a, b) ((a) > (b) ? (a) : (b))
#define MIN_VEC(V) *std::min_element(V.begin(), V.end())
#define MAX_VEC(V) *std::max_element(V.begin(), V.end())
#define LOG2(X) (size_t) std::ceil(std::log2((X)))
