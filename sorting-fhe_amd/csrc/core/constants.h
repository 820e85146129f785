// Forwarding header: OpenFHE's pke constants.h (PKESchemeFeature,
// ScalingTechnique, KeySwitchTechnique, ...), which the reference's
// tests/BitonicSortTest.cpp includes; the engine's openfhe.h declares them.
#pragma once
#include "openfhe.h"
