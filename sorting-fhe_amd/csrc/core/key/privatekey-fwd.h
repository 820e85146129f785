// Forwarding header: the reference includes OpenFHE's key/privatekey-fwd.h; the engine's
// facade declares everything in openfhe.h.
#pragma once
#include "openfhe.h"
