#include "lgap/threading.h"

#include <omp.h>

#include <mutex>

namespace lgap {

namespace {
std::mutex g_mu;
int g_default = -1;
int g_max = -1;
int g_omp_default = 0;  // OpenMP's team size before the library changed it

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
}

void SetMaxNumThreads(int num_threads) {
  std::lock_guard<std::mutex> lk(g_mu);
  (void)Effective();
  g_max = num_threads > 0 ? num_threads : -1;
  omp_set_num_threads(Effective());
}

void ApplyNumThreads() {
  int n;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_default <= 0 && g_max <= 0) return;  // nothing set: OpenMP's own default stays
    n = Effective();
  }
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
