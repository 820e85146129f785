// Forwarding header: the reference includes this OpenFHE path; everything it
// needs is declared by the engine's openfhe.h.
#pragma once
#include "openfhe.h"
