// Host Montgomery arithmetic of zk_host.hpp (finish_host, batch conversions, twiddle seeds):
// prints seeded products, squares, sums and differences of every field -- through the portable
// CIOS / SOS code and, when the CPU has ADX + BMI2, through the MULX/ADCX/ADOX products -- as hex
// lines that tests/test_native.py checks against Python big-integer arithmetic.
#include "zk_host.hpp"
#include <cstdio>
#include <random>
using namespace zkh;

template <class F>
static void hex(const Fe<F> &a) {
  for (int i = F::N - 1; i >= 0; i--) printf("%016llx", (unsigned long long)a.v[i]);
}
template <class F>
static void field(const char *name, std::mt19937_64 &g) {
  printf("field %s %d ", name, F::N);
  Fe<F> p;
  for (int i = 0; i < F::N; i++) p.v[i] = F::P[i];
  hex(p);
  printf("\n");
  for (int it = 0; it < 400; it++) {
    Fe<F> a, b;
    for (int i = 0; i < F::N; i++) { a.v[i] = g(); b.v[i] = g(); }
    // canonical operands, including the extremes 0, 1, p - 1, p - 2
    a.v[F::N - 1] %= F::P[F::N - 1];
    b.v[F::N - 1] %= F::P[F::N - 1];
    if (it < 4) for (int i = 0; i < F::N; i++) a.v[i] = i == 0 ? F::P[0] - 1 - (it & 1) : F::P[i];
    if (it == 4) set_zero(a);
    if (it == 5) { set_zero(b); b.v[0] = 1; }
    Fe<F> m, s, x, y, ma;
    mul_cios(m, a, b);
    sqr_sos(s, a);
    add(x, a, b);
    sub(y, a, b);
    printf("v ");
    hex(a); printf(" "); hex(b); printf(" "); hex(m); printf(" "); hex(s); printf(" "); hex(x); printf(" "); hex(y);
    if (cpu_has_adx()) {
      mul_adx(ma, a, b);
      printf(" "); hex(ma);
    }
    printf("\n");
  }
}
int main() {
  std::mt19937_64 g(20261017);
  field<BLS_Fp>("bls12_381_fp", g);
  field<BLS_Fr>("bls12_381_fr", g);
  field<BN_Fp>("bn128_fp", g);
  field<BN_Fr>("bn128_fr", g);
  printf("adx %d\n", cpu_has_adx() ? 1 : 0);
}
