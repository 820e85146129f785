// Forwarding header: the reference includes OpenFHE's key/key-ser.h; the engine's
// facade declares everything in openfhe.h.
#pragma once
#include "openfhe.h"
