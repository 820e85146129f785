// Composite sign approximation: public surface of the reference's src/sign.h
// (SignFunc sign.h:6-11, CompositeSignConfig :13-18, SignConfig :20-32,
// compositeSign<n> :35-38, sign() :40-41), implemented in sign.cpp on the
// device engine.
#pragma once

#include "encryption.h"
#include "openfhe.h"

enum class SignFunc {
    CompositeSign,
    SignumPolycircuit,
    Tanh,
    NaiveDiscrete,
};

// Composite polynomial g_n applied dg times, then f_n applied df times
// (Cheon-Kim-Kim, "Efficient Homomorphic Comparison Methods with Optimal
// Complexity", eprint 2019/1234).
struct CompositeSignConfig {
    int n;
    int dg;
    int df;
    CompositeSignConfig(int n, int dg, int df) : n(n), dg(dg), df(df) {}
};

struct SignConfig {
    CompositeSignConfig compos;
    // Depth budget used by the lazy-bootstrap rule; 100 = "never bootstrap".
    int multDepth;

    SignConfig() : compos(0, 0, 0), multDepth(100) {}
    SignConfig(CompositeSignConfig c) : compos(c.n, c.dg, c.df), multDepth(100) {}
    SignConfig(CompositeSignConfig c, int depth) : compos(c.n, c.dg, c.df), multDepth(depth) {}
};

template <int n>
lbcrypto::Ciphertext<lbcrypto::DCRTPoly> compositeSign(lbcrypto::Ciphertext<lbcrypto::DCRTPoly> x,
                                                       lbcrypto::CryptoContext<lbcrypto::DCRTPoly> cc,
                                                       const SignConfig& Cfg);

lbcrypto::Ciphertext<lbcrypto::DCRTPoly> sign(lbcrypto::Ciphertext<lbcrypto::DCRTPoly> x,
                                              lbcrypto::CryptoContext<lbcrypto::DCRTPoly> cc,
                                              SignFunc func, const SignConfig& Cfg);
