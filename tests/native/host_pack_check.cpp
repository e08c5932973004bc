// CPU check of csrc/host_pack.hpp (tests/test_host_pack.py): random tensors
// packed into staging rows by PackJob + PackPool at several thread counts,
// byte-compared with a plain concatenation; every unit must complete and the
// dispatcher sees units in order. Exit code 0 = pass.
#include <cstdio>
#include <random>
#include <vector>

#include "host_pack.hpp"

int main(int argc, char** argv) {
  const unsigned seed = argc > 1 ? static_cast<unsigned>(std::atoi(argv[1])) : 1u;
  std::mt19937_64 rng(seed);
  for (int trial = 0; trial < 40; ++trial) {
    const int n = 1 + static_cast<int>(rng() % 9), t = 1 + static_cast<int>(rng() % 40);
    std::vector<size_t> sz(t);
    size_t total = 0;
    for (auto& s : sz) {
      s = rng() % 5 == 0 ? rng() % 9 : rng() % (rng() % 3 == 0 ? 300000 : 5000);
      total += s;
    }
    const size_t esz = rng() % 2 ? 4 : 2, stride = (total + 7) / 8 * 8 + 8 * (rng() % 3);
    std::vector<std::vector<char>> src(static_cast<size_t>(n) * t);
    for (size_t j = 0; j < src.size(); ++j) {
      src[j].resize(sz[j % t] * esz + 1);  // +1: sources need no alignment
      for (auto& c : src[j]) c = static_cast<char>(rng());
    }
    const size_t shift = rng() % 2;  // unaligned source starts
    std::vector<char> stage(n * stride * esz + 64, 0), want(stage.size(), 0);
    char* base = stage.data() + (16 - (reinterpret_cast<uintptr_t>(stage.data()) & 15)) % 16;
    const size_t chunk = rng() % 3 == 0 ? total : 1024 * (1 + rng() % 64);
    const size_t n_chunks = total ? (total + chunk - 1) / chunk : 0;
    dlsim::PackJob job;
    std::vector<size_t> off(t + 1, 0);
    for (int k = 0; k < t; ++k) off[k + 1] = off[k] + sz[k];
    for (size_t c = 0; c < n_chunks; ++c) {
      const size_t c0 = c * chunk, c1 = std::min(total, c0 + chunk);
      for (int i = 0; i < n; ++i)
        for (int k = 0; k < t; ++k) {
          const size_t a = std::max(c0, off[k]), b = std::min(c1, off[k + 1]);
          if (a < b)
            job.add(static_cast<uint32_t>(c * n + i), src[i * t + k].data() + shift + (a - off[k]) * esz,
                    base + i * stride * esz + a * esz, (b - a) * esz);
        }
    }
    job.seal(n_chunks * n);
    const int helpers = static_cast<int>(rng() % 8);
    dlsim::PackPool& pool = dlsim::PackPool::get();
    std::vector<size_t> order;
    {
      std::lock_guard<std::mutex> lk(pool.call_mutex());
      if (helpers) pool.start(&job, helpers);
      for (size_t u = 0; u < job.units;) {
        if (job.unit_done(u)) order.push_back(u++);
        else if (!job.run_one()) std::this_thread::yield();
      }
      if (helpers) pool.join();
    }
    for (size_t u = 0; u < order.size(); ++u)
      if (order[u] != u) { std::printf("FAIL order trial %d\n", trial); return 1; }
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < t; ++k)
        if (sz[k] && std::memcmp(base + (i * stride + off[k]) * esz, src[i * t + k].data() + shift, sz[k] * esz)) {
          std::printf("FAIL bytes trial %d model %d tensor %d\n", trial, i, k);
          return 1;
        }
  }
  std::printf("OK\n");
  return 0;
}
