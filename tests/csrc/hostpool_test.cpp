// CPU test of pmvs_hostpool.h (tests/test_hostpool.py): every index of a range is visited exactly once
// for any thread count, concurrent callers either run on the pool or are told to run alone, and a
// forked child (none of the parent's workers) is told to run alone instead of waiting forever.
#include <sys/wait.h>

#include <atomic>
#include <cstdio>
#include <vector>

#include "pmvs_hostpool.h"

using pmvsdev::HostPool;

static int cover(int n, int nt) {  // 0: every index visited once
  std::vector<std::atomic<int>> hit(n);
  for (auto& h : hit) h = 0;
  const bool pooled = HostPool::get().run(nt, [&](int t, int k) {
    const int per = (n + k - 1) / k;
    for (int i = t * per; i < std::min(n, (t + 1) * per); ++i) hit[i]++;
  });
  if (!pooled) return 100;
  for (int i = 0; i < n; ++i)
    if (hit[i] != 1) return 1;
  return 0;
}

extern "C" int hostpool_check() {
  for (int rep = 0; rep < 200; ++rep)
    for (int nt : {1, 2, 3, 8, 64})
      if (int e = cover(1000 + rep, nt)) return e;
  // concurrent callers: each either gets the pool or runs alone; all indices still visited once
  std::atomic<int> bad{0}, alone{0};
  std::vector<std::thread> th;
  for (int c = 0; c < 4; ++c)
    th.emplace_back([&] {
      for (int rep = 0; rep < 100; ++rep) {
        const int n = 5000;
        std::vector<std::atomic<int>> hit(n);
        for (auto& h : hit) h = 0;
        auto body = [&](int t, int k) {
          const int per = (n + k - 1) / k;
          for (int i = t * per; i < std::min(n, (t + 1) * per); ++i) hit[i]++;
        };
        if (!HostPool::get().run(8, body)) {
          alone++;
          body(0, 1);
        }
        for (int i = 0; i < n; ++i)
          if (hit[i] != 1) bad++;
      }
    });
  for (auto& t : th) t.join();
  if (bad) return 2;
  // a forked child: run() must decline (the workers are the parent's)
  const pid_t pid = fork();
  if (pid == 0) _exit(HostPool::get().run(4, [](int, int) {}) ? 3 : 0);
  int status = 0;
  waitpid(pid, &status, 0);
  if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) return 3;
  return 0;
}
