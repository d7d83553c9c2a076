// Native unit / integration tests of the C++ core, the analogue of the reference's
// tests/cpp_tests (test_single_row.cpp, test_stream.cpp, test_serialize.cpp,
// test_common.cpp): plain asserts, no framework. Built by `make cpptest`
// (build/test_native) and `make asan` (build/asan/test_native, host code under
// AddressSanitizer + UBSan); tests/test_native.py runs whichever exist.
//
//   test_native <path to tests/data>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "lgap/c_api.h"
#include "lgap/common.h"
#include "lgap/pointwise_metric.h"
#include "lgap/random.h"
#include "lgap/split_math.h"
#include "learner/leaf_constraints.h"

namespace {

int g_failures = 0;

#define EXPECT(cond)                                                              \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::fprintf(stderr, "%s:%d: EXPECT failed: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                               \
    }                                                                             \
  } while (0)

#define CHECK_API(call) EXPECT((call) == 0)

std::vector<std::vector<double>> LoadTsv(const std::string& path, std::vector<float>* label) {
  std::ifstream in(path);
  std::string line;
  std::vector<std::vector<double>> rows;
  while (std::getline(in, line)) {
    std::stringstream ss(line);
    double v;
    std::vector<double> r;
    bool first = true;
    while (ss >> v) {
      if (first) label->push_back(static_cast<float>(v));
      else r.push_back(v);
      first = false;
    }
    if (!r.empty()) rows.push_back(r);
  }
  return rows;
}

void TestRandom() {
  // the reference LCG stream (random.h:101-111): x = 214013 x + 2531011
  lgap::Random r(7);
  unsigned x = 7u;
  for (int i = 0; i < 100; ++i) {
    x = 214013u * x + 2531011u;
    const float expect = static_cast<float>((x >> 16) & 0x7FFF) / 32768.0f;
    EXPECT(r.NextFloat() == expect);
  }
  lgap::Random s(3);
  const auto sample = s.Sample(100, 10);
  EXPECT(sample.size() == 10u);
  for (size_t i = 1; i < sample.size(); ++i) EXPECT(sample[i] > sample[i - 1]);
}

void TestCommon() {
  const auto parts = lgap::common::Split("a,b,,c", ',');
  EXPECT(parts.size() >= 3u);
  double d = 0.0;
  EXPECT(lgap::common::AtofOrDie("1.5e3") == 1500.0);
  (void)d;
  const std::vector<int> cats = {1, 5, 33, 64};
  const auto bits = lgap::common::ConstructBitset(cats.data(), static_cast<int>(cats.size()));
  EXPECT(bits.size() == 3u);
  EXPECT((bits[0] >> 1) & 1u);
  EXPECT((bits[0] >> 5) & 1u);
  EXPECT((bits[1] >> 1) & 1u);
  EXPECT((bits[2] >> 0) & 1u);
  EXPECT(!((bits[0] >> 2) & 1u));
}

void TestPointwiseMetric() {
  lgap::PwMetricParams p;
  p.kind = lgap::kPmBinLogloss;
  p.output = lgap::kOutSigmoid;
  p.sigmoid = 1.0;
  const double t = lgap::PmRowTerm(p, 1.0, 0.0, false, 1.0);
  EXPECT(std::fabs(t - std::log(2.0)) < 1e-12);
  p.kind = lgap::kPmL2;
  p.output = lgap::kOutIdentity;
  EXPECT(lgap::PmRowTerm(p, 2.0, 5.0, true, 0.5) == 4.5);
}

void TestTrainPredictRoundTrip(const std::string& data) {
  std::vector<float> y;
  const auto rows = LoadTsv(data + "/binary.test", &y);
  EXPECT(!rows.empty());
  if (rows.empty()) return;
  const int ncol = static_cast<int>(rows[0].size());
  DatasetHandle ds = nullptr;
  CHECK_API(LGBM_DatasetCreateFromFile((data + "/binary.train").c_str(), "max_bin=63 verbosity=-1", nullptr, &ds));
  int n = 0;
  CHECK_API(LGBM_DatasetGetNumData(ds, &n));
  EXPECT(n == 7000);
  BoosterHandle b = nullptr;
  CHECK_API(LGBM_BoosterCreate(ds, "objective=binary num_leaves=15 verbosity=-1 device_type=cpu", &b));
  int finished = 0;
  for (int it = 0; it < 20 && !finished; ++it) CHECK_API(LGBM_BoosterUpdateOneIter(b, &finished));

  // batch predictions vs single-row fast path (test_single_row.cpp)
  std::vector<double> flat;
  for (const auto& r : rows) flat.insert(flat.end(), r.begin(), r.end());
  const int nr = static_cast<int>(rows.size());
  std::vector<double> batch(nr);
  int64_t len = 0;
  CHECK_API(LGBM_BoosterPredictForMat(b, flat.data(), C_API_DTYPE_FLOAT64, nr, ncol, 1, C_API_PREDICT_NORMAL, 0, -1,
                                      "", &len, batch.data()));
  EXPECT(len == nr);
  FastConfigHandle fc = nullptr;
  CHECK_API(LGBM_BoosterPredictForMatSingleRowFastInit(b, C_API_PREDICT_NORMAL, 0, -1, C_API_DTYPE_FLOAT64, ncol, "",
                                                       &fc));
  for (int i = 0; i < nr; i += 37) {
    double out = 0.0;
    CHECK_API(LGBM_BoosterPredictForMatSingleRowFast(fc, rows[i].data(), &len, &out));
    EXPECT(std::fabs(out - batch[i]) < 1e-12);
  }
  CHECK_API(LGBM_FastConfigFree(fc));

  // model text round trip (test_serialize.cpp analogue for the model)
  int64_t need = 0;
  CHECK_API(LGBM_BoosterSaveModelToString(b, 0, -1, 0, 0, &need, nullptr));
  std::string text(static_cast<size_t>(need), '\0');
  CHECK_API(LGBM_BoosterSaveModelToString(b, 0, -1, 0, need, &need, &text[0]));
  BoosterHandle b2 = nullptr;
  int iters = 0;
  CHECK_API(LGBM_BoosterLoadModelFromString(text.c_str(), &iters, &b2));
  EXPECT(iters == 20);
  std::vector<double> again(nr);
  CHECK_API(LGBM_BoosterPredictForMat(b2, flat.data(), C_API_DTYPE_FLOAT64, nr, ncol, 1, C_API_PREDICT_NORMAL, 0, -1,
                                      "", &len, again.data()));
  for (int i = 0; i < nr; ++i) EXPECT(again[i] == batch[i]);
  double acc = 0.0;
  for (int i = 0; i < nr; ++i) acc += ((batch[i] > 0.5) == (y[i] > 0.5)) ? 1.0 : 0.0;
  EXPECT(acc / nr > 0.7);
  CHECK_API(LGBM_BoosterFree(b2));
  CHECK_API(LGBM_BoosterFree(b));

  // streaming push rows into a dataset created by reference (test_stream.cpp)
  DatasetHandle st = nullptr;
  CHECK_API(LGBM_DatasetCreateByReference(ds, nr, &st));
  const int half = nr / 2;
  CHECK_API(LGBM_DatasetPushRows(st, flat.data(), C_API_DTYPE_FLOAT64, half, ncol, 0));
  CHECK_API(LGBM_DatasetPushRows(st, flat.data() + static_cast<size_t>(half) * ncol, C_API_DTYPE_FLOAT64, nr - half,
                                 ncol, half));
  int sn = 0;
  CHECK_API(LGBM_DatasetGetNumData(st, &sn));
  EXPECT(sn == nr);
  CHECK_API(LGBM_DatasetFree(st));
  CHECK_API(LGBM_DatasetFree(ds));
}

// Errors raised inside OpenMP regions (parsing) must come back as -1 + LGBM_GetLastError,
// never std::terminate (reference utils/openmp_wrapper.h:80-131).
void TestParallelErrorsReturnMinusOne() {
  const std::string dir = "/tmp";
  const std::string bad_csv = dir + "/lgap_native_bad.csv";
  {
    std::ofstream f(bad_csv);
    for (int i = 0; i < 20000; ++i) {
      if (i == 12345) f << "1,2.5,oops,4\n";
      else f << (i % 2) << "," << i * 0.5 << "," << (i % 7) << "," << (i % 3) << "\n";
    }
  }
  DatasetHandle ds = nullptr;
  EXPECT(LGBM_DatasetCreateFromFile(bad_csv.c_str(), "verbosity=-1", nullptr, &ds) == -1);
  EXPECT(std::strstr(LGBM_GetLastError(), "oops") != nullptr);
  EXPECT(LGBM_DatasetCreateFromFile(bad_csv.c_str(), "verbosity=-1 two_round=true", nullptr, &ds) == -1);
  EXPECT(std::strstr(LGBM_GetLastError(), "oops") != nullptr);
  // a bad label token (label column parsed inside the same region)
  const std::string bad_label = dir + "/lgap_native_badlabel.csv";
  {
    std::ofstream f(bad_label);
    for (int i = 0; i < 20000; ++i) f << (i == 777 ? "yes" : (i % 2 ? "1" : "0")) << "," << i << "," << i % 5 << "\n";
  }
  EXPECT(LGBM_DatasetCreateFromFile(bad_label.c_str(), "verbosity=-1", nullptr, &ds) == -1);
  EXPECT(std::strstr(LGBM_GetLastError(), "yes") != nullptr);
  // a query file whose sizes do not add up to the row count
  const std::string good = dir + "/lgap_native_rank.csv";
  {
    std::ofstream f(good);
    for (int i = 0; i < 1000; ++i) f << (i % 3) << "," << i << "," << i % 5 << "\n";
    std::ofstream q(good + ".query");
    q << "500\n400\n";
  }
  EXPECT(LGBM_DatasetCreateFromFile(good.c_str(), "verbosity=-1", nullptr, &ds) == -1);
  EXPECT(std::strlen(LGBM_GetLastError()) > 0);
  std::remove(bad_csv.c_str());
  std::remove(bad_label.c_str());
  std::remove(good.c_str());
  std::remove((good + ".query").c_str());
}

}  // namespace

// Piecewise per-bin bounds of the advanced monotone method against a dense per-bin
// model (reference monotone_constraints.hpp:872-965 UpdateConstraints semantics:
// a leaf output tightens the bound on the bin range [b, e) it shares).
void TestBinPiecesMatchDenseBounds() {
  lgap::Random r(7);
  for (int trial = 0; trial < 400; ++trial) {
    const int nb = 2 + r.NextShort(0, 60);
    const bool raise = trial & 1;
    lgap::BinPieces p;
    p.Reset(raise ? -INFINITY : INFINITY);
    std::vector<double> dense(nb, raise ? -INFINITY : INFINITY);
    for (int op = 0; op < 12; ++op) {
      const double v = r.NextShort(-8, 8) * 0.25;
      if (r.NextShort(0, 5) == 0) {
        p.TightenAll(v, raise);
        for (double& x : dense) x = raise ? std::max(x, v) : std::min(x, v);
        continue;
      }
      const uint32_t b = r.NextShort(0, nb), e = b + 1 + r.NextShort(0, nb);
      p.TightenRange(v, raise, b, e, nb);
      for (uint32_t t = b; t < std::min<uint32_t>(e, nb); ++t) dense[t] = raise ? std::max(dense[t], v) : std::min(dense[t], v);
    }
    std::vector<double> got(nb);
    p.Expand(nb, got.data());
    for (int t = 0; t < nb; ++t) EXPECT(got[t] == dense[t]);
    EXPECT(p.start[0] == 0);
    for (size_t i = 1; i < p.size(); ++i) EXPECT(p.start[i] > p.start[i - 1] && p.val[i] != p.val[i - 1]);
  }
}

int main(int argc, char** argv) {
  const std::string data = argc > 1 ? argv[1] : "tests/data";
  TestRandom();
  TestCommon();
  TestPointwiseMetric();
  TestTrainPredictRoundTrip(data);
  TestParallelErrorsReturnMinusOne();
  TestBinPiecesMatchDenseBounds();
  if (g_failures) {
    std::fprintf(stderr, "%d expectation(s) failed\n", g_failures);
    return 1;
  }
  std::printf("test_native: all passed\n");
  return 0;
}
