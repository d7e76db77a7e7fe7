// Host check of zk_inv.hpp (the device inversion's code, compiled for the CPU): prints
// "<field> <x> <x^-1>" lines in hex for tests/test_native.py to verify with Python big integers.
#include <stdio.h>
#include <stdint.h>
#include <random>
#include "zk_inv.hpp"
#include "zk_params.inc"

template <int L, int NB, int B = 62>
static void run(const char *name, const int64_t (&P)[L], uint64_t pinv, int n64, const uint64_t *pw, int count,
                std::mt19937_64 &rng) {
  for (int k = 0; k < count; k++) {
    uint64_t x[6] = {0, 0, 0, 0, 0, 0}, y[6];
    if (k == 0) x[0] = 1;
    else if (k == 1) {  // p - 1
      for (int i = 0; i < n64; i++) x[i] = pw[i];
      x[0] -= 1;
    } else if (k == 2) x[0] = 2;
    else if (k == 3) x[0] = 0;  // 0 -> 0
    else {
      for (int i = 0; i < n64; i++) x[i] = rng();
      // reduce below p by clearing the top bits beyond p's top word and subtracting p while >= p
      int top = 63;
      while (!((pw[n64 - 1] >> top) & 1)) top--;
      x[n64 - 1] &= (top == 63) ? ~0ull : ((1ull << (top + 1)) - 1);
      for (;;) {
        int ge = 1;
        for (int i = n64 - 1; i >= 0; i--) {
          if (x[i] != pw[i]) { ge = x[i] > pw[i]; break; }
        }
        if (!ge) break;
        uint64_t br = 0;
        for (int i = 0; i < n64; i++) {
          const uint64_t a = x[i], b = pw[i] + br;
          br = (b < br) || (a < b);
          x[i] = a - b;
        }
      }
    }
    zk::sg_inverse_words<L, NB, B>(y, x, n64, P, pinv);
    printf("%s ", name);
    for (int i = n64 - 1; i >= 0; i--) printf("%016llx", (unsigned long long)x[i]);
    printf(" ");
    for (int i = n64 - 1; i >= 0; i--) printf("%016llx", (unsigned long long)y[i]);
    printf("\n");
  }
}

int main() {
  std::mt19937_64 rng(12345);
  {
    static const int64_t P[] = ZK_BLS12_381_FP_S62_P;
    const uint64_t pw[6] = {0xb9feffffffffaaabull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                            0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
    static const int64_t P60[] = ZK_BLS12_381_FP_S60_P;
    run<ZK_BLS12_381_FP_S60_L, ZK_BLS12_381_FP_S60_BATCHES, 60>("bls12_381_fp", P60, ZK_BLS12_381_FP_S62_PINV, 6, pw, 1000, rng);
    run<ZK_BLS12_381_FP_S62_L, ZK_BLS12_381_FP_S62_BATCHES>("bls12_381_fp", P, ZK_BLS12_381_FP_S62_PINV, 6, pw,
                                                            2000, rng);
  }
  {
    static const int64_t P[] = ZK_BLS12_381_FR_S62_P;
    const uint64_t pw[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                            0x73eda753299d7d48ull};
    static const int64_t P60[] = ZK_BLS12_381_FR_S60_P;
    run<ZK_BLS12_381_FR_S60_L, ZK_BLS12_381_FR_S60_BATCHES, 60>("bls12_381_fr", P60, ZK_BLS12_381_FR_S62_PINV, 4, pw, 1000, rng);
    run<ZK_BLS12_381_FR_S62_L, ZK_BLS12_381_FR_S62_BATCHES>("bls12_381_fr", P, ZK_BLS12_381_FR_S62_PINV, 4, pw,
                                                            2000, rng);
  }
  {
    static const int64_t P[] = ZK_BN128_FP_S62_P;
    const uint64_t pw[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull,
                            0x30644e72e131a029ull};
    static const int64_t P60[] = ZK_BN128_FP_S60_P;
    run<ZK_BN128_FP_S60_L, ZK_BN128_FP_S60_BATCHES, 60>("bn128_fp", P60, ZK_BN128_FP_S62_PINV, 4, pw, 1000, rng);
    run<ZK_BN128_FP_S62_L, ZK_BN128_FP_S62_BATCHES>("bn128_fp", P, ZK_BN128_FP_S62_PINV, 4, pw, 2000, rng);
  }
  {
    static const int64_t P[] = ZK_BN128_FR_S62_P;
    const uint64_t pw[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                            0x30644e72e131a029ull};
    static const int64_t P60[] = ZK_BN128_FR_S60_P;
    run<ZK_BN128_FR_S60_L, ZK_BN128_FR_S60_BATCHES, 60>("bn128_fr", P60, ZK_BN128_FR_S62_PINV, 4, pw, 1000, rng);
    run<ZK_BN128_FR_S62_L, ZK_BN128_FR_S62_BATCHES>("bn128_fr", P, ZK_BN128_FR_S62_PINV, 4, pw, 2000, rng);
  }
  return 0;
}
