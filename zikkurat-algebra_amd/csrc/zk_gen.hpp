// zk_gen.hpp -- deterministic synthetic input generator (spec in zk_gen.cpp)
#pragma once
#include <stdint.h>
namespace zkg {
template <class F> void gen_field(uint64_t seed, int64_t start, int64_t count, uint64_t *out);
template <class Fp, class Fr>
void gen_points(uint64_t seed, int64_t start, int64_t count, uint64_t *out, const uint64_t *gx, const uint64_t *gy,
                const uint64_t *b3);
}  // namespace zkg
