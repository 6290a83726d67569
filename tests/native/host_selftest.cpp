// Host-side logic of libmini_nccl under AddressSanitizer + UBSan (sanitizers
// on host code only -- GPU ASan is not available on the test pool).  Built and run by
// tests/test_host_sanitizers.py with g++ -fsanitize=address,undefined; exercises the code
// the GPU path shares with the CPU simulator: csrc/schedule.h index math (through sim.cpp's
// kernel-mirroring programs: the ring and both forms of read), the TCP bootstrap (threads over 127.0.0.1),
// the read schedule's shared-memory call board (csrc/peerbuf.cpp) and env config parsing.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <thread>
#include <vector>

extern "C" {
int mnccl_sim_allreduce(uint64_t algo, const float* const* send, float* const* recv, int n, uint64_t count, int op,
                        uint64_t slice_bytes, uint64_t min_slice, int channels, int slots, int calls,
                        uint64_t schedule_seed, uint64_t* steps_out);
int mnccl_bootstrap_selftest(int rank, int nranks, const char* ip, int port, int timeout_ms);
int mnccl_config_describe(char* buf, int len);
int mnccl_board_selftest(int rank, int nranks, const char* ip, int port, int scenario, int calls, double timeout_s,
                         int* decisions);
}

static int sim_case(int algo, int n, uint64_t count, uint64_t slice, uint64_t min_slice, int channels, int slots,
                    int calls, uint64_t seed) {
  std::mt19937 g((unsigned)(seed * 7 + n));
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  std::vector<std::vector<float>> s((size_t)n, std::vector<float>(count)), r((size_t)n, std::vector<float>(count));
  for (auto& v : s)
    for (auto& x : v) x = u(g);
  std::vector<const float*> sp;
  std::vector<float*> rp;
  for (int i = 0; i < n; ++i) {
    sp.push_back(s[(size_t)i].data());
    rp.push_back(r[(size_t)i].data());
  }
  uint64_t steps = 0;
  uint64_t mask = 0;  // 3 bits per call: the schedule of every call (tests/sim_api.py codes)
  for (int c = 0; c < calls; ++c) mask |= (uint64_t)algo << (3 * c);
  const int rc = mnccl_sim_allreduce(mask, sp.data(), rp.data(), n, count, 0, slice, min_slice, channels, slots, calls,
                                     seed, &steps);
  if (rc != 0) return 1;
  // every rank holds the same bits in the body (the count % n tail keeps each rank's own
  // input; the oracle comparison lives in the Python tests)
  const uint64_t body = count / (uint64_t)n * (uint64_t)n;
  for (int i = 1; i < n; ++i)
    for (uint64_t k = 0; k < body; ++k)
      if (r[(size_t)i][k] != r[0][k] && !(r[(size_t)i][k] != r[(size_t)i][k])) return 2;
  return 0;
}

int main() {
  int fails = 0;
  const uint64_t counts[] = {7, 1000, 4099, 70001};
  for (int algo : {0, 2, 4})  // ring, read (persistent kernel), read's grid form
    for (int n = 2; n <= 8; n += 3)
      for (uint64_t c : counts)
        for (int adaptive = 0; adaptive < 2; ++adaptive) {
          const int rc = sim_case(algo, n, c, 256, adaptive ? 64 : 0, 3, 2 + (int)(c % 2), 2, c + (uint64_t)n);
          if (rc) {
            printf("sim FAIL algo=%d n=%d count=%llu adaptive=%d rc=%d\n", algo, n, (unsigned long long)c, adaptive, rc);
            ++fails;
          }
        }
  // the one-shot schedule: a slot holds n pieces, so a larger slot and 64 pipelines
  for (int n = 2; n <= 8; n += 3)
    for (uint64_t c : counts)
      for (int adaptive = 0; adaptive < 2; ++adaptive) {
        const int rc = sim_case(1, n, c, 16384, adaptive ? 64 : 0, 64, 2 + (int)(c % 2), 3, c + (uint64_t)n);
        if (rc) {
          printf("sim FAIL one-shot n=%d count=%llu adaptive=%d rc=%d\n", n, (unsigned long long)c, adaptive, rc);
          ++fails;
        }
      }
  // bootstrap: 3 ranks as threads over loopback
  const char* pe = getenv("SELFTEST_PORT");
  const int port = pe ? atoi(pe) : 29471;
  std::vector<int> rcs(3, -9);
  std::vector<std::thread> th;
  for (int r = 0; r < 3; ++r) th.emplace_back([&, r] { rcs[(size_t)r] = mnccl_bootstrap_selftest(r, 3, "127.0.0.1", port, 20000); });
  for (auto& t : th) t.join();
  for (int r = 0; r < 3; ++r)
    if (rcs[(size_t)r] != 0) {
      printf("bootstrap FAIL rank %d rc=%d\n", r, rcs[(size_t)r]);
      ++fails;
    }
  // the read schedule's call board: 3 ranks as threads, 40 calls with a count mismatch at call 20
  {
    std::vector<std::vector<int>> dec(3, std::vector<int>(40, -7));
    std::vector<int> brc(3, -9);
    std::vector<std::thread> bt;
    for (int r = 0; r < 3; ++r)
      bt.emplace_back([&, r] { brc[(size_t)r] = mnccl_board_selftest(r, 3, "127.0.0.1", port + 1, 1, 40, 10.0, dec[(size_t)r].data()); });
    for (auto& t : bt) t.join();
    for (int r = 0; r < 3; ++r) {
      bool ok = brc[(size_t)r] == 0;
      for (int i = 0; i < 40; ++i) ok = ok && dec[(size_t)r][(size_t)i] == (i == 20 ? -1 : 0);
      if (!ok) {
        printf("board FAIL rank %d rc=%d\n", r, brc[(size_t)r]);
        ++fails;
      }
    }
  }
  // the board's mapping round: 3 ranks as threads, synthetic buffers, rank 1 fails to map on
  // call 3 -> that call falls back on every rank, every other call reads (decision + 10 x rounds)
  {
    std::vector<std::vector<int>> dec(3, std::vector<int>(24, -7));
    std::vector<int> brc(3, -9);
    std::vector<std::thread> bt;
    for (int r = 0; r < 3; ++r)
      bt.emplace_back([&, r] { brc[(size_t)r] = mnccl_board_selftest(r, 3, "127.0.0.1", port + 2, 4, 24, 10.0, dec[(size_t)r].data()); });
    for (auto& t : bt) t.join();
    for (int r = 0; r < 3; ++r) {
      bool ok = brc[(size_t)r] == 0;
      for (int i = 0; i < 24; ++i) ok = ok && dec[(size_t)r][(size_t)i] == (i == 2 ? 0 : 1) + 10 * (i + 1);
      if (!ok) {
        printf("mapping round FAIL rank %d rc=%d\n", r, brc[(size_t)r]);
        ++fails;
      }
    }
  }
  char buf[512];
  if (mnccl_config_describe(buf, (int)sizeof buf) != 0) {
    printf("config FAIL: %s\n", buf);
    ++fails;
  }
  printf("host selftest: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
