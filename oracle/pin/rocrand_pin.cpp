// rocrand_pin.cpp - TEST INFRASTRUCTURE ONLY (oracle pin, see cvr_oracle.c).
//
// cuRAND's XORWOW (used by the reference through Rng.h:22,26) is not in this
// image, so its output cannot be checked here.  rocRAND ships the same
// generator (Marsaglia's xorwow with Weyl sequence, rocrand_xorwow.h
// xorwow_engine::next) with different seeding constants and a different
// float mapping.  This program loads a state (v0..v4, d) given on the command
// line into rocRAND's engine and prints its next() outputs, so that the
// oracle's state-transition function can be checked against an independent
// implementation (tests/test_oracle_cpu.py).
//
//   rocrand_pin v0 v1 v2 v3 v4 d n   -> n decimal u32 values, one per line
//   rocrand_pin seed S               -> rocRAND's state after xorwow_engine(S, 0, 0): v0..v4 d
//                                       (pins the oracle's seeding structure, rng_init_consts)
#include <rocrand/rocrand_xorwow.h>

#include <cstdio>
#include <cstdlib>
#include <string>

struct pinned_xorwow : rocrand_device::xorwow_engine {
  pinned_xorwow(const unsigned (&v)[5], unsigned d) : xorwow_engine(0ull, 0ull, 0ull) {
    for (int i = 0; i < 5; ++i) m_state.x[i] = v[i];
    m_state.d = d;
  }
};

struct seeded_xorwow : rocrand_device::xorwow_engine {
  explicit seeded_xorwow(unsigned long long seed) : xorwow_engine(seed, 0ull, 0ull) {}
  void print() const {
    for (int i = 0; i < 5; ++i) std::printf("%u\n", m_state.x[i]);
    std::printf("%u\n", m_state.d);
  }
};

int main(int argc, char** argv) {
  if (argc == 3 && std::string(argv[1]) == "seed") {
    seeded_xorwow(std::strtoull(argv[2], nullptr, 10)).print();
    return 0;
  }
  if (argc != 8) {
    std::fprintf(stderr, "usage: %s v0 v1 v2 v3 v4 d n\n", argv[0]);
    return 2;
  }
  unsigned v[5];
  for (int i = 0; i < 5; ++i) v[i] = (unsigned)std::strtoul(argv[1 + i], nullptr, 10);
  const unsigned d = (unsigned)std::strtoul(argv[6], nullptr, 10);
  const long n = std::strtol(argv[7], nullptr, 10);
  pinned_xorwow e(v, d);
  for (long i = 0; i < n; ++i) std::printf("%u\n", e.next());
  return 0;
}
