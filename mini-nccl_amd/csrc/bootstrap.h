// bootstrap.h -- TCP rendezvous for the communicator's one-time exchange.
//
// Plays the role of the reference's rank-0 star (RDMATransport.h:516-593 over
// Socket.h:31-107): rank 0 listens on ip:port, the others connect (bounded retries),
// and fixed-size records are all-gathered through rank 0.  The reference also ran
// this exchange on EVERY all-reduce (exchange_dynamic_info, RDMATransport.h:171-257);
// here it runs only in ncclCommInitRank / ncclCommDestroy: the hot path never touches
// the host network.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string>
#include <vector>

namespace mnccl {

class Bootstrap {
 public:
  Bootstrap() = default;
  ~Bootstrap();
  Bootstrap(const Bootstrap&) = delete;
  Bootstrap& operator=(const Bootstrap&) = delete;

  // Throws std::runtime_error on failure (bind/connect/timeout).
  void connect(int rank, int nranks, const std::string& ip, int port, double timeout_s);
  // all-gather of `bytes` per rank: out receives nranks * bytes, rank-major
  void allgather(const void* mine, void* out, size_t bytes);
  void barrier();
  void close_all();

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }

 private:
  static void send_all(int fd, const void* p, size_t n);
  static void recv_all(int fd, void* p, size_t n, double timeout_s);
  int rank_ = -1, nranks_ = 0;
  double timeout_s_ = 60.0;
  std::vector<int> clients_;  // rank 0: fd per rank (index = rank; [0] unused)
  int root_fd_ = -1;          // ranks > 0: connection to rank 0
};

}  // namespace mnccl
