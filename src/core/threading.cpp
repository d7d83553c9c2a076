#include "lgap/threading.h"

#include <omp.h>

#include <atomic>
#include <mutex>

namespace lgap {

namespace {
std::mutex g_mu;
int g_default = -1;
int g_max = -1;
int g_omp_default = 0;  // OpenMP's team size before the library changed it
// the team size every API entry applies (-1: nothing set, OpenMP's default stays); written under
// g_mu by the setters, read lock-free by ApplyNumThreads (hot single-row predict paths)
std::atomic<int> g_apply{-1};

int Effective() {
  if (g_omp_default <= 0) g_omp_default = omp_get_max_threads();
  int n = g_default > 0 ? g_default : g_omp_default;
  if (g_max > 0 && n > g_max) n = g_max;
  return n;
}
}  // namespace

void SetDefaultNumThreads(int num_threads) {
  std::lock_guard<std::mutex> lk(g_mu);
  (void)Effective();
  g_default = num_threads > 0 ? num_threads : -1;
  omp_set_num_threads(Effective());
  g_apply.store(g_default <= 0 && g_max <= 0 ? -1 : Effective(), std::memory_order_release);
}

void SetMaxNumThreads(int num_threads) {
  std::lock_guard<std::mutex> lk(g_mu);
  (void)Effective();
  g_max = num_threads > 0 ? num_threads : -1;
  omp_set_num_threads(Effective());
  g_apply.store(g_default <= 0 && g_max <= 0 ? -1 : Effective(), std::memory_order_release);
}

void ApplyNumThreads() {
  const int n = g_apply.load(std::memory_order_acquire);
  if (n <= 0) return;  // nothing set: OpenMP's own default stays
  if (omp_get_max_threads() != n) omp_set_num_threads(n);
}

int MaxNumThreadsSetting() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_max;
}

int NumThreads() {
  std::lock_guard<std::mutex> lk(g_mu);
  return Effective();
}

}  // namespace lgap
