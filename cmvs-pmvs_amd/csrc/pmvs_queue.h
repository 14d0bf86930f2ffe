// pmvs_queue.h -- CExpand's max-_tmp priority queue on the host, as sorted runs.  The reference's is a
// std::priority_queue of patches under P_compare (expand.hpp:31, patchOrganizerS.hpp:10-15: by _tmp;
// the order of equal _tmp is left to the heap), popped at expand.cpp:82-86 and pushed at
// expand.cpp:251; here equal _tmp pop in push order (the key's low half), so the schedule is
// deterministic.  Host code only: included by pmvs_filter.hip and by the CPU test
// tests/csrc/run_queue_test.cpp.
#pragma once
#include <algorithm>
#include <cstring>
#include <utility>
#include <vector>

namespace pmvsdev {

struct QItem {
  unsigned long long key;
  int p;
};
static inline unsigned long long qkey(float tmp, long long seq) {
  if (tmp == 0.0f) tmp = 0.0f;
  unsigned u;
  std::memcpy(&u, &tmp, sizeof(u));
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (0xffffffffull - (unsigned long long)seq);
}
struct QCmp {  // max-heap on key
  bool operator()(const QItem& a, const QItem& b) const { return a.key < b.key; }
};
// CExpand's max-_tmp queue as sorted runs: the collected patches (one run, sorted on the device)
// and one run per wave (the patches that wave pushed, in key order); a pop takes the largest run
// head through a max-heap over the runs (at most a few hundred: log2 of them per pop instead of a
// binary heap over every queued patch).  Keys are unique (seq), so the pops are the same sequence
// a single heap over all items gives.
class RunQueue {
 public:
  bool empty() const { return heads_.empty(); }
  // r sorted by key, descending
  void add_run(std::vector<QItem>&& r) {
    if (r.empty()) return;
    const int id = (int)runs_.size();
    runs_.push_back(std::move(r));
    pos_.push_back(0);
    heads_.push_back({runs_[id][0].key, id});
    std::push_heap(heads_.begin(), heads_.end());
  }
  int pop() {
    std::pop_heap(heads_.begin(), heads_.end());
    const int id = heads_.back().second;
    heads_.pop_back();
    std::vector<QItem>& r = runs_[id];
    const int p = r[pos_[id]].p;
    if (++pos_[id] < r.size()) {
      heads_.push_back({r[pos_[id]].key, id});
      std::push_heap(heads_.begin(), heads_.end());
    } else {
      std::vector<QItem>().swap(r);
    }
    return p;
  }
  // up to k pops appended to out, the same sequence as k pop() calls: the top run gives items while
  // its head stays above every other run's head (one heap step per stretch instead of per item)
  size_t pop_many(std::vector<int>& out, size_t k) {
    size_t got = 0;
    while (got < k && !heads_.empty()) {
      std::pop_heap(heads_.begin(), heads_.end());
      const int id = heads_.back().second;
      heads_.pop_back();
      const bool others = !heads_.empty();
      const unsigned long long next = others ? heads_.front().first : 0ull;
      std::vector<QItem>& r = runs_[id];
      size_t i = pos_[id];
      do {
        out.push_back(r[i].p);
        ++i;
        ++got;
      } while (got < k && i < r.size() && (!others || r[i].key > next));
      pos_[id] = i;
      if (i < r.size()) {
        heads_.push_back({r[i].key, id});
        std::push_heap(heads_.begin(), heads_.end());
      } else {
        std::vector<QItem>().swap(r);
      }
    }
    return got;
  }
  // a wave's pushes, in push order (seq ascending = low key bits descending): a stable LSD radix sort
  // on the high 32 key bits (the _tmp order bits), descending, gives the run's key order
  static void sort_run(std::vector<QItem>& v, std::vector<QItem>& tmp) {
    const size_t n = v.size();
    tmp.resize(n);
    for (int sh = 32; sh < 64; sh += 8) {
      size_t cnt[257] = {0};
      for (const QItem& q : v) cnt[255 - ((q.key >> sh) & 0xff) + 1]++;
      for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
      for (const QItem& q : v) tmp[cnt[255 - ((q.key >> sh) & 0xff)]++] = q;
      v.swap(tmp);
    }
  }

 private:
  std::vector<std::vector<QItem>> runs_;
  std::vector<size_t> pos_;
  std::vector<std::pair<unsigned long long, int>> heads_;
};

}  // namespace pmvsdev
