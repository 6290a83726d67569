// bootstrap.cpp -- see bootstrap.h.
#include "bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace mnccl {

namespace {

double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

bool resolve(const std::string& host, int port, sockaddr_in* out) {
  memset(out, 0, sizeof *out);
  out->sin_family = AF_INET;
  out->sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &out->sin_addr) == 1) return true;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return false;
  out->sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return true;
}

// Handshake record sent by every non-root rank right after connecting.
struct Hello {
  uint32_t magic;  // 'MNCC'
  int32_t rank;
  int32_t nranks;
};
constexpr uint32_t kMagic = 0x4d4e4343u;

}  // namespace

Bootstrap::~Bootstrap() { close_all(); }

void Bootstrap::close_all() {
  for (int fd : clients_)
    if (fd >= 0) ::close(fd);
  clients_.clear();
  if (root_fd_ >= 0) ::close(root_fd_);
  root_fd_ = -1;
}

void Bootstrap::send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) throw std::runtime_error(std::string("bootstrap send failed: ") + strerror(errno));
    c += k;
    n -= (size_t)k;
  }
}

void Bootstrap::recv_all(int fd, void* p, size_t n, double timeout_s) {
  char* c = static_cast<char*>(p);
  const double deadline = now_s() + timeout_s;
  while (n) {
    pollfd pf{fd, POLLIN, 0};
    const double left = deadline - now_s();
    if (left <= 0) throw std::runtime_error("bootstrap recv timed out");
    int pr = ::poll(&pf, 1, (int)(left * 1000) + 1);
    if (pr < 0 && errno == EINTR) continue;
    if (pr <= 0) throw std::runtime_error("bootstrap recv timed out");
    ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) throw std::runtime_error("bootstrap peer closed the connection");
    c += k;
    n -= (size_t)k;
  }
}

void Bootstrap::connect(int rank, int nranks, const std::string& ip, int port, double timeout_s) {
  rank_ = rank;
  nranks_ = nranks;
  timeout_s_ = timeout_s;
  if (nranks == 1) return;
  const double deadline = now_s() + timeout_s;
  if (rank == 0) {
    int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (lfd < 0) throw std::runtime_error("bootstrap: socket() failed");
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    a.sin_port = htons((uint16_t)port);
    if (::bind(lfd, reinterpret_cast<sockaddr*>(&a), sizeof a) < 0 || ::listen(lfd, 256) < 0) {
      const std::string e = strerror(errno);
      ::close(lfd);
      throw std::runtime_error("bootstrap: cannot listen on port " + std::to_string(port) + ": " + e);
    }
    clients_.assign((size_t)nranks, -1);
    int joined = 0;
    try {
      while (joined < nranks - 1) {
        const double left = deadline - now_s();
        if (left <= 0) throw std::runtime_error("bootstrap: timed out waiting for ranks to connect");
        pollfd pf{lfd, POLLIN, 0};
        int pr = ::poll(&pf, 1, (int)(left * 1000) + 1);
        if (pr < 0 && errno == EINTR) continue;
        if (pr <= 0) continue;
        int fd = ::accept(lfd, nullptr, nullptr);
        if (fd < 0) continue;
        set_nodelay(fd);
        Hello h{};
        recv_all(fd, &h, sizeof h, left);
        if (h.magic != kMagic || h.nranks != nranks || h.rank <= 0 || h.rank >= nranks || clients_[(size_t)h.rank] >= 0) {
          ::close(fd);
          throw std::runtime_error("bootstrap: bad or duplicate hello (rank " + std::to_string(h.rank) + ", nranks " +
                                   std::to_string(h.nranks) + ")");
        }
        clients_[(size_t)h.rank] = fd;
        ++joined;
      }
    } catch (...) {
      ::close(lfd);
      throw;
    }
    ::close(lfd);
  } else {
    sockaddr_in a;
    if (!resolve(ip, port, &a)) throw std::runtime_error("bootstrap: cannot resolve " + ip);
    for (;;) {
      int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (fd < 0) throw std::runtime_error("bootstrap: socket() failed");
      if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) == 0) {
        set_nodelay(fd);
        root_fd_ = fd;
        break;
      }
      ::close(fd);
      if (now_s() > deadline)
        throw std::runtime_error("bootstrap: cannot connect to " + ip + ":" + std::to_string(port));
      usleep(50 * 1000);
    }
    Hello h{kMagic, rank, nranks};
    send_all(root_fd_, &h, sizeof h);
  }
}

void Bootstrap::allgather(const void* mine, void* out, size_t bytes) {
  char* o = static_cast<char*>(out);
  memcpy(o + (size_t)rank_ * bytes, mine, bytes);
  if (nranks_ == 1) return;
  if (rank_ == 0) {
    for (int r = 1; r < nranks_; ++r) recv_all(clients_[(size_t)r], o + (size_t)r * bytes, bytes, timeout_s_);
    for (int r = 1; r < nranks_; ++r) send_all(clients_[(size_t)r], o, bytes * (size_t)nranks_);
  } else {
    send_all(root_fd_, mine, bytes);
    recv_all(root_fd_, o, bytes * (size_t)nranks_, timeout_s_);
  }
}

void Bootstrap::barrier() {
  char b = 1;
  std::vector<char> all((size_t)nranks_);
  allgather(&b, all.data(), 1);
}

}  // namespace mnccl
