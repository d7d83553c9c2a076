// Exception transport out of OpenMP regions.
//
// An exception may not leave an OpenMP structured block: one thrown by
// Log::Fatal inside `#pragma omp parallel` would call std::terminate and kill
// the host process (breaking the C API's "-1 + LGBM_GetLastError" contract).
// Every parallel loop whose body can throw catches into an OmpErrors and the
// serial code after the region rethrows the first captured exception, so the
// error surfaces as if the loop had run serially. After a failure the other
// iterations are skipped cheaply. Role of the reference's
// include/LightGBM/utils/openmp_wrapper.h:80-131 (OMP_INIT_EX / OMP_LOOP_EX_* /
// OMP_THROW_EX), written as a small class instead of macros.
//
//   OmpErrors errs;
//   #pragma omp parallel for
//   for (int i = 0; i < n; ++i) {
//     if (errs.failed()) continue;
//     try { Body(i); } catch (...) { errs.Capture(); }
//   }
//   errs.Rethrow();
#pragma once

#include <atomic>
#include <exception>
#include <mutex>

namespace lgap {

class OmpErrors {
 public:
  // called from a catch(...) block inside the region
  void Capture() noexcept {
    std::lock_guard<std::mutex> lock(mu_);
    if (!first_) first_ = std::current_exception();
    failed_.store(true, std::memory_order_relaxed);
  }
  bool failed() const noexcept { return failed_.load(std::memory_order_relaxed); }
  // called after the region, from the thread that entered it
  void Rethrow() {
    if (!failed()) return;
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> lock(mu_);
      e = first_;
      first_ = nullptr;
      failed_.store(false, std::memory_order_relaxed);
    }
    if (e) std::rethrow_exception(e);
  }
  // Runs f() with capture; for loop bodies written as lambdas.
  template <typename F>
  void Run(F&& f) noexcept {
    if (failed()) return;
    try {
      f();
    } catch (...) {
      Capture();
    }
  }

 private:
  std::mutex mu_;
  std::exception_ptr first_;
  std::atomic<bool> failed_{false};
};

}  // namespace lgap
