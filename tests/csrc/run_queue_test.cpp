// CPU test of pmvs_queue.h (tests/test_run_queue.py): the sorted-run queue pops the same sequence as
// one binary heap (std::priority_queue under QCmp) over the same keys, for random waves of pushes
// with many equal _tmp values, interleaved with batch pops (single pops and pop_many).
#include <cstdio>
#include <queue>
#include <random>

#include "pmvs_queue.h"

using namespace pmvsdev;

extern "C" int run_queue_check(unsigned seed, int nwaves, int initial, long long* npops) {
  std::mt19937 rng(seed);
  std::uniform_int_distribution<int> tmpi(-3, 40);  // few distinct values: many ties
  std::uniform_int_distribution<int> wsz(0, 3000), popn(1, 4000);
  std::priority_queue<QItem, std::vector<QItem>, QCmp> heap;
  RunQueue rq;
  long long seq = 0;
  std::vector<QItem> run, tmp;
  for (int i = 0; i < initial; ++i) run.push_back({qkey(tmpi(rng) * 0.25f, seq++), i});
  for (const QItem& q : run) heap.push(q);
  RunQueue::sort_run(run, tmp);  // the device sorts the initial run; here the same order by the host sort
  rq.add_run(std::vector<QItem>(run));
  int pid = initial;
  *npops = 0;
  for (int w = 0; w < nwaves; ++w) {
    const int np = popn(rng);
    if (w & 1) {  // odd waves: one pop_many call (the expansion's), the same sequence as np pops
      std::vector<int> got;
      const size_t n = rq.pop_many(got, (size_t)np);
      if (n != got.size()) return 5;
      for (size_t k = 0; k < n; ++k) {
        if (heap.empty()) return 6;
        const int a = heap.top().p;
        heap.pop();
        if (a != got[k]) return 2;
        ++*npops;
      }
      if (n < (size_t)np && !heap.empty()) return 7;
    } else {
      for (int k = 0; k < np && !heap.empty(); ++k) {
        if (rq.empty()) return 1;
        const int a = heap.top().p;
        heap.pop();
        const int b = rq.pop();
        if (a != b) return 2;
        ++*npops;
      }
    }
    run.clear();
    const int ns = wsz(rng);
    for (int k = 0; k < ns; ++k) {
      const float t = (k % 7 == 0) ? -0.0f : tmpi(rng) * 0.25f;
      run.push_back({qkey(t, seq++), pid++});
    }
    for (const QItem& q : run) heap.push(q);
    RunQueue::sort_run(run, tmp);
    rq.add_run(std::vector<QItem>(run));
  }
  while (!heap.empty()) {
    if (rq.empty()) return 3;
    const int a = heap.top().p;
    heap.pop();
    if (a != rq.pop()) return 4;
    ++*npops;
  }
  return rq.empty() ? 0 : 5;
}
