// pmvs_hostcomm.cpp -- a host all-gather over TCP for multi-process pmvs2 jobs.
//
// The cluster exchange (pmvs_scene_set_cluster) needs an all-gather between the ranks of one job.
// On an 8-GPU node the records travel device to device over RCCL (pmvs_rccl.cpp); this channel is
// the job's bootstrap and its host-memory fallback:
//   * pmvs2 ranks find each other through the torchrun-style environment (MASTER_ADDR, MASTER_PORT,
//     RANK, WORLD_SIZE): rank 0 listens, the others connect (star);
//   * rank 0's RCCL unique id reaches every rank through one all-gather on it;
//   * with PMVS_EXCHANGE=tcp the boundary records themselves go through it -- several ranks on ONE
//     GPU (RCCL refuses two ranks per device), e.g. the two-process test of tests/test_gpu_pmvs2.py.
// One all-gather: every rank sends {bytes, data} to rank 0, which checks that the sizes agree and
// returns {status, world x data, commit} to each (commit 0: every peer was served).  A peer that dies closes its socket, so its partners'
// reads fail and the exchange returns -1 instead of blocking (the loop's error protocol then ends
// every rank).  Blocking reads without a time limit: an exchange waits for the slowest rank's
// expansion, which may take minutes.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/pmvs_amd.h"

pmvs_status pmvs_io_fail(pmvs_status st, const char* fmt, ...);  // pmvs_api.cpp: sets pmvs_last_error

struct pmvs_tcp {
  int rank = 0, world = 1;
  int hub = -1;               // rank > 0: the connection to rank 0
  std::vector<int> peers;     // rank 0: the connection of rank r at peers[r] (peers[0] = -1)
};

namespace {

bool write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

// read_all with a time limit (the join handshake: a client that connects and sends nothing must not
// hold rank 0 past the job's start-up deadline)
bool read_all_within(int fd, void* p, size_t n, int ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
  char* c = static_cast<char*>(p);
  while (n) {
    const long long left =
        std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count();
    pollfd pf{fd, POLLIN, 0};
    const int pr = ::poll(&pf, 1, (int)std::max<long long>(0, left));
    if (pr < 0 && errno == EINTR) continue;
    if (pr <= 0) return false;
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool drain(int fd, size_t n) {
  char buf[4096];
  while (n) {
    const size_t k = n < sizeof(buf) ? n : sizeof(buf);
    if (!read_all(fd, buf, k)) return false;
    n -= k;
  }
  return true;
}

void tune(int fd) {
  int one = 1;
  (void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

bool resolve(const char* addr, int port, sockaddr_in* sa) {
  std::memset(sa, 0, sizeof(*sa));
  sa->sin_family = AF_INET;
  sa->sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, addr, &sa->sin_addr) == 1) return true;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(addr, nullptr, &hints, &res) != 0 || !res) return false;
  sa->sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return true;
}

constexpr uint32_t kMagic = 0x504d5653;  // "PMVS": a stray connection is refused

}  // namespace

pmvs_status pmvs_tcp_create(int32_t rank, int32_t world, const char* addr, int32_t port, int32_t timeout_ms,
                            pmvs_tcp** out) {
  if (!out || !addr || world < 1 || rank < 0 || rank >= world || port <= 0 || port > 65535 || timeout_ms < 0)
    return pmvs_io_fail(PMVS_EINVAL, "invalid tcp arguments");
  *out = nullptr;
  sockaddr_in sa;
  if (!resolve(addr, port, &sa)) return pmvs_io_fail(PMVS_EINVAL, "cannot resolve %s", addr);
  auto* c = new pmvs_tcp();
  c->rank = rank;
  c->world = world;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  auto left_ms = [&]() {
    return (int)std::max<long long>(
        0, std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count());
  };
  if (world == 1) {
    *out = c;
    return PMVS_OK;
  }
  if (rank == 0) {
    const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    (void)setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (ls < 0 || ::bind(ls, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(ls, world) != 0) {
      if (ls >= 0) ::close(ls);
      delete c;
      return pmvs_io_fail(PMVS_EDEVICE, "tcp: cannot listen on %s:%d (%s)", addr, port, std::strerror(errno));
    }
    c->peers.assign(world, -1);
    int joined = 1;
    while (joined < world) {
      pollfd pf{ls, POLLIN, 0};
      const int pr = ::poll(&pf, 1, left_ms());
      if (pr <= 0) {
        ::close(ls);
        pmvs_tcp_destroy(c);
        return pmvs_io_fail(PMVS_EDEVICE, "tcp: %d of %d ranks joined within %d ms", joined, world, timeout_ms);
      }
      const int fd = ::accept(ls, nullptr, nullptr);
      if (fd < 0) continue;
      uint32_t hello[3] = {0, 0, 0};  // magic, rank, world
      if (!read_all_within(fd, hello, sizeof(hello), left_ms()) || hello[0] != kMagic || hello[2] != (uint32_t)world || hello[1] == 0 ||
          hello[1] >= (uint32_t)world || c->peers[hello[1]] >= 0) {
        ::close(fd);
        continue;
      }
      tune(fd);
      c->peers[hello[1]] = fd;
      ++joined;
    }
    ::close(ls);
  } else {
    while (true) {
      const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (fd >= 0 && ::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) == 0) {
        const uint32_t hello[3] = {kMagic, (uint32_t)rank, (uint32_t)world};
        if (write_all(fd, hello, sizeof(hello))) {
          tune(fd);
          c->hub = fd;
          break;
        }
      }
      if (fd >= 0) ::close(fd);
      if (left_ms() == 0) {
        delete c;
        return pmvs_io_fail(PMVS_EDEVICE, "tcp: rank %d cannot reach %s:%d within %d ms", rank, addr, port, timeout_ms);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
  }
  *out = c;
  return PMVS_OK;
}

void pmvs_tcp_destroy(pmvs_tcp* c) {
  if (!c) return;
  if (c->hub >= 0) ::close(c->hub);
  for (int fd : c->peers)
    if (fd >= 0) ::close(fd);
  delete c;
}

int pmvs_tcp_allgather(void* ctx, const void* send, int64_t bytes, void* recv) {
  auto* c = static_cast<pmvs_tcp*>(ctx);
  if (!c || bytes < 0) return -1;
  const size_t b = (size_t)bytes;
  if (c->world == 1) {
    if (b) std::memcpy(recv, send, b);
    return 0;
  }
  if (c->rank > 0) {
    const int64_t h = bytes;
    if (!write_all(c->hub, &h, sizeof(h)) || (b && !write_all(c->hub, send, b))) return -1;
    int32_t status = -1;
    if (!read_all(c->hub, &status, sizeof(status))) return -1;
    if (status == 0 && b && !read_all(c->hub, recv, b * (size_t)c->world)) return -1;
    // the commit word, sent after every exchange (so a failed one leaves the stream in step): 0 only
    // if rank 0 delivered the payload to every peer
    int32_t commit = -1;
    if (!read_all(c->hub, &commit, sizeof(commit))) return -1;
    return (status == 0 && commit == 0) ? 0 : -1;
  }
  // rank 0: collect, check, broadcast.  A peer that is gone (or sends a different size) fails the
  // exchange for everyone: the live peers still get the failure status, so none of them blocks.
  int32_t status = 0;
  char* r = static_cast<char*>(recv);
  if (b) std::memcpy(r, send, b);
  for (int p = 1; p < c->world; ++p) {
    int& fd = c->peers[p];
    int64_t h = -1;
    if (fd < 0 || !read_all(fd, &h, sizeof(h))) {
      if (fd >= 0) ::close(fd);
      fd = -1;
      status = -1;
      continue;
    }
    if (h != bytes) {
      status = -1;
      if (h > 0 && !drain(fd, (size_t)h)) { ::close(fd); fd = -1; }
      continue;
    }
    if (b && !read_all(fd, r + (size_t)p * b, b)) {
      ::close(fd);
      fd = -1;
      status = -1;
    }
  }
  // status to every peer first, then the payload to every peer that was told 0, then a commit word:
  // a peer returns success only if every peer was served.  A peer told 0 always gets its payload, even
  // when a later peer fails, so it never waits for bytes that do not come; the commit word is decided
  // before any is sent, so every live rank returns the same outcome.  A peer whose write fails is
  // closed, which fails its own read (and every later exchange).
  // PMVS_TEST_TCP_FAIL=p:k (tests only): the status write to peer p fails in this rank's k-th exchange.
  static int inj_peer = -2, inj_call = 0, calls = 0;
  if (inj_peer == -2) {
    inj_peer = -1;
    if (const char* e = getenv("PMVS_TEST_TCP_FAIL")) (void)sscanf(e, "%d:%d", &inj_peer, &inj_call);
  }
  ++calls;
  std::vector<int32_t> told(c->world, -1);
  for (int p = 1; p < c->world; ++p) {
    int& fd = c->peers[p];
    if (fd < 0) continue;
    const bool fail = (p == inj_peer && calls == inj_call);
    if (fail || !write_all(fd, &status, sizeof(status))) {
      ::close(fd);
      fd = -1;
      status = -1;
    } else {
      told[p] = status;
    }
  }
  if (b)
    for (int p = 1; p < c->world; ++p) {
      int& fd = c->peers[p];
      if (fd < 0 || told[p] != 0) continue;
      if (!write_all(fd, r, b * (size_t)c->world)) { ::close(fd); fd = -1; status = -1; }
    }
  int32_t commit = status;
  for (int p = 1; p < c->world; ++p)
    if (c->peers[p] < 0 || told[p] != 0) commit = -1;
  for (int p = 1; p < c->world; ++p) {
    int& fd = c->peers[p];
    if (fd < 0) continue;
    if (!write_all(fd, &commit, sizeof(commit))) { ::close(fd); fd = -1; }
  }
  return commit == 0 ? 0 : -1;
}
