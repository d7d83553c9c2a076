// LGBM_* C ABI (reference: src/c_api.cpp:47-3000). The Booster wrapper guards
// training with a unique lock and prediction / evaluation with a shared lock
// (c_api.cpp:54-58). Exceptions become -1 + LGBM_GetLastError.
#include "lgap/omp_errors.h"
#include "lgap/threading.h"
#include "lgap/c_api.h"
#include "lgap/parser.h"

#include <omp.h>

#include <algorithm>
#include <cstring>
#include <functional>
#include <fstream>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <sstream>
#include <string>
#include <vector>

#include "lgap/arrow.h"
#include "lgap/boosting.h"
#include "lgap/common.h"
#include "lgap/config.h"
#include "lgap/dataset.h"
#include "lgap/device_api.h"
#include "lgap/log.h"
#include "lgap/metric.h"
#include "lgap/network.h"
#include "lgap/objective.h"

using namespace lgap;

namespace {

thread_local std::string g_last_error = "Everything is fine";
void SetLastError(const char* msg) { g_last_error = msg; }

// Every entry point applies the library's thread setting to the CALLING thread's OpenMP team
// size (omp_set_num_threads is per-thread state): a Booster's num_threads and
// LGBM_SetMaxThreads hold whichever host thread trains or predicts (Python threads, joblib,
// Dask workers), as the reference's num_threads(OMP_NUM_THREADS()) on every region does.
#define API_BEGIN() \
  try {             \
    ::lgap::ApplyNumThreads();
#define API_END()                      \
  }                                    \
  catch (std::exception & ex) {        \
    SetLastError(ex.what());           \
    return -1;                         \
  }                                    \
  catch (...) {                        \
    SetLastError("unknown exception"); \
    return -1;                         \
  }                                    \
  return 0;

void CopyStr(const std::string& s, int64_t buffer_len, int64_t* out_len, char* out) {
  *out_len = static_cast<int64_t>(s.size()) + 1;
  if (out != nullptr && buffer_len >= *out_len) std::memcpy(out, s.c_str(), s.size() + 1);
}

void CopyStrings(const std::vector<std::string>& v, int len, int* out_len, size_t buffer_len, size_t* out_buffer_len,
                 char** out) {
  *out_len = static_cast<int>(v.size());
  *out_buffer_len = 0;
  for (int i = 0; i < static_cast<int>(v.size()); ++i) {
    *out_buffer_len = std::max(*out_buffer_len, v[i].size() + 1);
    if (i < len && out != nullptr && out[i] != nullptr) {
      std::memcpy(out[i], v[i].c_str(), std::min(buffer_len, v[i].size() + 1));
      if (buffer_len > 0) out[i][buffer_len - 1] = out[i][buffer_len - 1];
    }
  }
}

Config ParseConfig(const char* params) {
  Config c;
  c.Set(Config::Str2Map(params ? params : ""));
  SetDefaultNumThreads(c.num_threads);  // reference c_api.cpp OMP_SET_NUM_THREADS(config.num_threads)
  return c;
}

std::vector<int> CategoricalIndices(const Config& c) {
  std::vector<int> out;
  if (c.categorical_feature.empty() || common::StartsWith(c.categorical_feature, "name:")) return out;
  for (auto& t : common::Split(c.categorical_feature, ',')) out.push_back(common::AtoiOrDie(t));
  return out;
}

// CSC -> rows
std::unique_ptr<OwnedSparseSource> CSCToRows(const void* col_ptr, int col_ptr_type, const int32_t* indices,
                                             const void* data, int data_type, int64_t ncol_ptr, int64_t num_row) {
  auto src = std::make_unique<OwnedSparseSource>();
  src->rows.resize(num_row);
  src->ncol = static_cast<int>(ncol_ptr - 1);
  for (int64_t c = 0; c + 1 < ncol_ptr; ++c) {
    int64_t b = col_ptr_type == C_API_DTYPE_INT64 ? static_cast<const int64_t*>(col_ptr)[c] : static_cast<const int32_t*>(col_ptr)[c];
    int64_t e = col_ptr_type == C_API_DTYPE_INT64 ? static_cast<const int64_t*>(col_ptr)[c + 1] : static_cast<const int32_t*>(col_ptr)[c + 1];
    for (int64_t k = b; k < e; ++k) {
      double v = data_type == C_API_DTYPE_FLOAT64 ? static_cast<const double*>(data)[k] : static_cast<const float*>(data)[k];
      src->rows[indices[k]].emplace_back(static_cast<int>(c), v);
    }
  }
  return src;
}

// Several dense matrices stacked by rows.
class MultiDenseSource : public RowSource {
 public:
  MultiDenseSource(std::vector<DenseSource> mats) : mats_(std::move(mats)) {
    for (auto& m : mats_) {
      starts_.push_back(total_);
      total_ += m.num_rows();
    }
  }
  data_size_t num_rows() const override { return total_; }
  int num_cols() const override { return mats_.empty() ? 0 : mats_[0].num_cols(); }
  void GetRow(data_size_t i, std::vector<std::pair<int, double>>* out) const override {
    size_t m = std::upper_bound(starts_.begin(), starts_.end(), i) - starts_.begin() - 1;
    mats_[m].GetRow(i - starts_[m], out);
  }

 private:
  std::vector<DenseSource> mats_;
  std::vector<data_size_t> starts_;
  data_size_t total_ = 0;
};

struct DatasetWrapper {
  std::unique_ptr<Dataset> ds;
  Config cfg;
  // field buffers returned by GetField
  std::vector<int32_t> group_buf;
};

class Booster {
 public:
  Booster(DatasetWrapper* train, const char* params) : train_(train) {
    auto pm = Config::Str2Map(params);
    config_.Set(pm);
    SetDefaultNumThreads(config_.num_threads);
    if (config_.num_machines > 1 && Network::num_machines() <= 1 && !config_.machines.empty()) {
      Network::Init(config_);
    }
    boosting_ = CreateBoosting(config_.boosting, nullptr);
    CreateObjectiveAndMetrics();
    boosting_->Init(&config_, train_->ds.get(), objective_.get(), MetricPtrs(train_metrics_));
  }
  explicit Booster(const char* model_str, size_t len) {
    boosting_ = CreateBoosting("gbdt", nullptr);
    if (!boosting_->LoadModelFromString(model_str, len)) Log::Fatal("Failed to load model");
  }

  void CreateObjectiveAndMetrics() {
    objective_ = ObjectiveFunction::Create(config_.objective, config_);
    if (objective_) objective_->Init(train_->ds->metadata(), train_->ds->num_data());
    train_metrics_.clear();
    for (auto& m : config_.metric) {
      auto met = Metric::Create(m, config_);
      if (!met) continue;
      met->Init(train_->ds->metadata(), train_->ds->num_data());
      train_metrics_.push_back(std::move(met));
    }
  }
  static std::vector<const Metric*> MetricPtrs(const std::vector<std::unique_ptr<Metric>>& v) {
    std::vector<const Metric*> out;
    for (auto& m : v) out.push_back(m.get());
    return out;
  }

  void AddValidData(DatasetWrapper* valid) {
    std::unique_lock<std::shared_mutex> lk(mu_);
    std::vector<std::unique_ptr<Metric>> ms;
    for (auto& m : config_.metric) {
      auto met = Metric::Create(m, config_);
      if (!met) continue;
      met->Init(valid->ds->metadata(), valid->ds->num_data());
      ms.push_back(std::move(met));
    }
    boosting_->AddValidDataset(valid->ds.get(), MetricPtrs(ms));
    valid_metrics_.push_back(std::move(ms));
  }

  bool TrainOneIter() {
    std::unique_lock<std::shared_mutex> lk(mu_);
    return boosting_->TrainOneIter(nullptr, nullptr);
  }
  bool TrainOneIterCustom(const float* g, const float* h) {
    std::unique_lock<std::shared_mutex> lk(mu_);
    return boosting_->TrainOneIter(g, h);
  }
  void ResetParameter(const char* params) {
    std::unique_lock<std::shared_mutex> lk(mu_);
    auto pm = Config::Str2Map(params);
    if (pm.count("num_class") && common::AtoiOrDie(pm["num_class"]) != config_.num_class) {
      Log::Fatal("Cannot change num_class during training");
    }
    // compared after parsing, so restating the current values is allowed (reference
    // c_api.cpp Booster::ResetConfig)
    Config next = config_;
    next.Set(pm);
    if (pm.count("boosting") && next.boosting != config_.boosting) Log::Fatal("Cannot change boosting during training");
    if (pm.count("metric") && next.metric != config_.metric) Log::Fatal("Cannot change metric during training");
    config_.Set(pm);
    SetDefaultNumThreads(config_.num_threads);
    if (pm.count("objective")) {
      objective_ = ObjectiveFunction::Create(config_.objective, config_);
      if (objective_) objective_->Init(train_->ds->metadata(), train_->ds->num_data());
    }
    boosting_->ResetConfig(&config_);
  }

  std::shared_mutex mu_;
  Config config_;
  DatasetWrapper* train_ = nullptr;
  std::unique_ptr<GBDT> boosting_;
  std::unique_ptr<ObjectiveFunction> objective_;
  std::vector<std::unique_ptr<Metric>> train_metrics_;
  std::vector<std::vector<std::unique_ptr<Metric>>> valid_metrics_;
};

Booster* B(BoosterHandle h) { return static_cast<Booster*>(h); }
DatasetWrapper* D(DatasetHandle h) { return static_cast<DatasetWrapper*>(h); }

// ---- prediction over a row source
void PredictRows(Booster* b, const RowSource& src, int predict_type, int start_iteration, int num_iteration,
                 const char* parameter, int64_t* out_len, double* out) {
  std::shared_lock<std::shared_mutex> lk(b->mu_);
  Config pc = ParseConfig(parameter);
  GBDT* g = b->boosting_.get();
  const bool leaf = predict_type == C_API_PREDICT_LEAF_INDEX;
  const bool contrib = predict_type == C_API_PREDICT_CONTRIB;
  const bool raw = predict_type == C_API_PREDICT_RAW_SCORE;
  g->InitPredict(start_iteration, num_iteration, contrib);
  const int per_row = g->NumPredictOneRow(start_iteration, num_iteration, leaf, contrib);
  const data_size_t n = src.num_rows();
  const int nf = std::max(g->MaxFeatureIdx() + 1, src.num_cols());
  if (!pc.predict_disable_shape_check && src.num_cols() != g->MaxFeatureIdx() + 1 && src.num_cols() > 0) {
    Log::Fatal("The number of features in data (%d) is not the same as it was in training data (%d).\n"
               "You can set ``predict_disable_shape_check=true`` to discard this error, but please be aware what you are doing.",
               src.num_cols(), g->MaxFeatureIdx() + 1);
  }
  // reference predictor.hpp:46-58: any objective that needs no accurate raw scores (binary,
  // multiclass, ranking) stops early; "binary" margins for one class, "multiclass" otherwise
  std::string es_type = "none";
  if (pc.pred_early_stop && !leaf && !contrib && !g->NeedAccuratePrediction()) {
    es_type = g->NumberOfClasses() == 1 ? "binary" : "multiclass";
  }
  PredictionEarlyStop es(es_type, pc.pred_early_stop_freq, pc.pred_early_stop_margin);
  OmpErrors errs;  // a failing row source (Arrow / Python callback) must return -1, not abort
#pragma omp parallel
  {
    std::vector<double> x(nf);
    std::vector<std::pair<int, double>> row;
#pragma omp for schedule(static)
    for (data_size_t i = 0; i < n; ++i) {
      errs.Run([&] {
        src.GetRow(i, &row);
        std::fill(x.begin(), x.end(), 0.0);
        for (auto& kv : row) if (kv.first < nf) x[kv.first] = kv.second;
        double* o = out + static_cast<size_t>(i) * per_row;
        if (leaf) g->PredictLeafIndex(x.data(), o);
        else if (contrib) g->PredictContrib(x.data(), o);
        else if (raw) g->PredictRaw(x.data(), o, &es);
        else g->Predict(x.data(), o, &es);
      });
    }
  }
  errs.Rethrow();
  *out_len = static_cast<int64_t>(n) * per_row;
}

}  // namespace

// ============================================================================
const char* LGBM_GetLastError() { return g_last_error.c_str(); }

int LGBM_RegisterLogCallback(void (*callback)(const char*)) {
  API_BEGIN();
  Log::ResetCallback(callback);
  API_END();
}

int LGBM_DumpParamAliases(int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  CopyStr(Config::DumpAliases(), buffer_len, out_len, out_str);
  API_END();
}

int LGBM_GetSampleCount(int32_t num_total_row, const char* parameters, int* out) {
  API_BEGIN();
  Config c = ParseConfig(parameters);
  *out = std::min(num_total_row, c.bin_construct_sample_cnt);
  API_END();
}

int LGBM_SampleIndices(int32_t num_total_row, const char* parameters, void* out, int32_t* out_len) {
  API_BEGIN();
  Config c = ParseConfig(parameters);
  Random r(c.data_random_seed);
  auto idx = r.Sample(num_total_row, std::min(num_total_row, c.bin_construct_sample_cnt));
  std::memcpy(out, idx.data(), idx.size() * sizeof(int32_t));
  *out_len = static_cast<int32_t>(idx.size());
  API_END();
}

// ---------------------------------------------------------------------------
int LGBM_DatasetCreateFromFile(const char* filename, const char* parameters, const DatasetHandle reference,
                               DatasetHandle* out) {
  API_BEGIN();
  auto w = std::make_unique<DatasetWrapper>();
  w->cfg = ParseConfig(parameters);
  w->ds = LoadDatasetFromFile(filename, w->cfg, reference ? D(reference)->ds.get() : nullptr, Network::rank(),
                              Network::num_machines());
  *out = w.release();
  API_END();
}

static DatasetHandle BuildFromSource(const RowSource& src, const char* parameters, const DatasetHandle reference) {
  auto w = std::make_unique<DatasetWrapper>();
  w->cfg = ParseConfig(parameters);
  w->ds = std::make_unique<Dataset>();
  w->ds->Construct(src, w->cfg, reference ? D(reference)->ds.get() : nullptr, {}, CategoricalIndices(w->cfg));
  return w.release();
}

int LGBM_DatasetCreateFromMat(const void* data, int data_type, int32_t nrow, int32_t ncol, int is_row_major,
                              const char* parameters, const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  DenseSource src(data, data_type == C_API_DTYPE_FLOAT64, nrow, ncol, is_row_major != 0);
  *out = BuildFromSource(src, parameters, reference);
  API_END();
}

int LGBM_DatasetCreateFromMats(int32_t nmat, const void** data, int data_type, int32_t* nrow, int32_t ncol,
                               int is_row_major, const char* parameters, const DatasetHandle reference,
                               DatasetHandle* out) {
  API_BEGIN();
  std::vector<DenseSource> mats;
  for (int i = 0; i < nmat; ++i) mats.emplace_back(data[i], data_type == C_API_DTYPE_FLOAT64, nrow[i], ncol, is_row_major != 0);
  MultiDenseSource src(std::move(mats));
  *out = BuildFromSource(src, parameters, reference);
  API_END();
}

int LGBM_DatasetCreateFromCSR(const void* indptr, int indptr_type, const int32_t* indices, const void* data,
                              int data_type, int64_t nindptr, int64_t nelem, int64_t num_col, const char* parameters,
                              const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  CSRSource src(indptr, indptr_type == C_API_DTYPE_INT64, indices, data, data_type == C_API_DTYPE_FLOAT64, nindptr,
                nelem, num_col);
  *out = BuildFromSource(src, parameters, reference);
  API_END();
}

int LGBM_DatasetCreateFromCSC(const void* col_ptr, int col_ptr_type, const int32_t* indices, const void* data,
                              int data_type, int64_t ncol_ptr, int64_t nelem, int64_t num_row, const char* parameters,
                              const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  (void)nelem;
  auto src = CSCToRows(col_ptr, col_ptr_type, indices, data, data_type, ncol_ptr, num_row);
  *out = BuildFromSource(*src, parameters, reference);
  API_END();
}

int LGBM_DatasetCreateByReference(const DatasetHandle reference, int64_t num_total_row, DatasetHandle* out) {
  API_BEGIN();
  auto w = std::make_unique<DatasetWrapper>();
  w->cfg = D(reference)->cfg;
  w->ds = std::make_unique<Dataset>();
  w->ds->InitEmptyLike(*D(reference)->ds, static_cast<data_size_t>(num_total_row));
  *out = w.release();
  API_END();
}

int LGBM_DatasetInitStreaming(DatasetHandle, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t) {
  API_BEGIN();
  API_END();
}

int LGBM_DatasetPushRows(DatasetHandle dataset, const void* data, int data_type, int32_t nrow, int32_t ncol,
                         int32_t start_row) {
  API_BEGIN();
  DenseSource src(data, data_type == C_API_DTYPE_FLOAT64, nrow, ncol, true);
  D(dataset)->ds->PushRows(src, start_row);
  API_END();
}

int LGBM_DatasetPushRowsWithMetadata(DatasetHandle dataset, const void* data, int data_type, int32_t nrow,
                                     int32_t ncol, int32_t start_row, const float* label, const float* weight,
                                     const double* init_score, const int32_t* query, int32_t) {
  API_BEGIN();
  DenseSource src(data, data_type == C_API_DTYPE_FLOAT64, nrow, ncol, true);
  Dataset* ds = D(dataset)->ds.get();
  ds->PushRows(src, start_row);
  ds->metadata().SetRows(start_row, nrow, label, weight, init_score, query);
  API_END();
}

int LGBM_DatasetPushRowsByCSR(DatasetHandle dataset, const void* indptr, int indptr_type, const int32_t* indices,
                              const void* data, int data_type, int64_t nindptr, int64_t nelem, int64_t num_col,
                              int64_t start_row) {
  API_BEGIN();
  CSRSource src(indptr, indptr_type == C_API_DTYPE_INT64, indices, data, data_type == C_API_DTYPE_FLOAT64, nindptr,
                nelem, num_col);
  D(dataset)->ds->PushRows(src, static_cast<data_size_t>(start_row));
  API_END();
}

int LGBM_DatasetSetWaitForManualFinish(DatasetHandle, int) {
  API_BEGIN();
  API_END();
}
int LGBM_DatasetMarkFinished(DatasetHandle) {
  API_BEGIN();
  API_END();
}

int LGBM_DatasetGetSubset(const DatasetHandle handle, const int32_t* used_row_indices, int32_t num_used_row_indices,
                          const char* parameters, DatasetHandle* out) {
  API_BEGIN();
  auto w = std::make_unique<DatasetWrapper>();
  w->cfg = ParseConfig(parameters);
  std::vector<data_size_t> idx(used_row_indices, used_row_indices + num_used_row_indices);
  w->ds = D(handle)->ds->Subset(idx);
  *out = w.release();
  API_END();
}

int LGBM_DatasetSetFeatureNames(DatasetHandle handle, const char** feature_names, int num_feature_names) {
  API_BEGIN();
  std::vector<std::string> n(feature_names, feature_names + num_feature_names);
  D(handle)->ds->set_feature_names(n);
  API_END();
}

int LGBM_DatasetGetFeatureNames(DatasetHandle handle, const int len, int* num_feature_names, const size_t buffer_len,
                                size_t* out_buffer_len, char** feature_names) {
  API_BEGIN();
  CopyStrings(D(handle)->ds->feature_names(), len, num_feature_names, buffer_len, out_buffer_len, feature_names);
  API_END();
}

int LGBM_DatasetFree(DatasetHandle handle) {
  API_BEGIN();
  delete D(handle);
  API_END();
}

int LGBM_DatasetSaveBinary(DatasetHandle handle, const char* filename) {
  API_BEGIN();
  D(handle)->ds->SaveBinary(filename);
  API_END();
}

int LGBM_DatasetDumpText(DatasetHandle handle, const char* filename) {
  API_BEGIN();
  const Dataset* ds = D(handle)->ds.get();
  std::ofstream out(filename);
  out << "num_features: " << ds->num_features() << "\nnum_groups: " << ds->num_groups() << "\n";
  out << "feature_names: " << common::Join(ds->feature_names(), ", ") << "\n";
  for (data_size_t i = 0; i < ds->num_data(); ++i) {
    for (int f = 0; f < ds->num_features(); ++f) out << (f ? ", " : "") << ds->FeatureBin(i, f);
    out << "\n";
  }
  API_END();
}

int LGBM_DatasetSetField(DatasetHandle handle, const char* field_name, const void* field_data, int num_element,
                         int type) {
  API_BEGIN();
  auto& md = D(handle)->ds->metadata();
  std::string name(field_name);
  if (name == "label" || name == "target") {
    if (type == C_API_DTYPE_FLOAT32) {
      md.SetLabel(static_cast<const float*>(field_data), num_element);
    } else {
      std::vector<float> v(num_element);
      for (int i = 0; i < num_element; ++i) v[i] = static_cast<float>(static_cast<const double*>(field_data)[i]);
      md.SetLabel(v.data(), num_element);
    }
  } else if (name == "weight" || name == "weights") {
    if (field_data == nullptr || num_element == 0) {
      md.SetWeights(nullptr, 0);
    } else if (type == C_API_DTYPE_FLOAT32) {
      md.SetWeights(static_cast<const float*>(field_data), num_element);
    } else {
      std::vector<float> v(num_element);
      for (int i = 0; i < num_element; ++i) v[i] = static_cast<float>(static_cast<const double*>(field_data)[i]);
      md.SetWeights(v.data(), num_element);
    }
  } else if (name == "init_score") {
    if (field_data == nullptr || num_element == 0) {
      md.SetInitScore(nullptr, 0);
    } else if (type == C_API_DTYPE_FLOAT64) {
      md.SetInitScore(static_cast<const double*>(field_data), num_element);
    } else {
      std::vector<double> v(num_element);
      for (int i = 0; i < num_element; ++i) v[i] = static_cast<const float*>(field_data)[i];
      md.SetInitScore(v.data(), num_element);
    }
  } else if (name == "group" || name == "query") {
    md.SetQuery(static_cast<const int32_t*>(field_data), num_element);
  } else if (name == "position") {
    md.SetPosition(static_cast<const int32_t*>(field_data), num_element);
  } else {
    Log::Fatal("Unknown field name: %s", field_name);
  }
  API_END();
}

int LGBM_DatasetGetField(DatasetHandle handle, const char* field_name, int* out_len, const void** out_ptr,
                         int* out_type) {
  API_BEGIN();
  auto* w = D(handle);
  auto& md = w->ds->metadata();
  std::string name(field_name);
  *out_ptr = nullptr;
  *out_len = 0;
  if (name == "label" || name == "target") {
    *out_ptr = md.label();
    *out_len = md.num_data();
    *out_type = C_API_DTYPE_FLOAT32;
  } else if (name == "weight" || name == "weights") {
    *out_ptr = md.weights();
    *out_len = md.weights() ? md.num_data() : 0;
    *out_type = C_API_DTYPE_FLOAT32;
  } else if (name == "init_score") {
    *out_ptr = md.init_score();
    *out_len = static_cast<int>(md.init_score_size());
    *out_type = C_API_DTYPE_FLOAT64;
  } else if (name == "group" || name == "query") {
    w->group_buf.assign(md.query_boundaries_vec().begin(), md.query_boundaries_vec().end());
    *out_ptr = w->group_buf.empty() ? nullptr : w->group_buf.data();
    *out_len = static_cast<int>(w->group_buf.size());
    *out_type = C_API_DTYPE_INT32;
  } else if (name == "position") {
    *out_ptr = md.positions();
    *out_len = md.positions() ? md.num_data() : 0;
    *out_type = C_API_DTYPE_INT32;
  } else {
    Log::Fatal("Unknown field name: %s", field_name);
  }
  API_END();
}

int LGBM_DatasetUpdateParamChecking(const char* old_parameters, const char* new_parameters) {
  API_BEGIN();
  // only the binning / loading parameters given in `new_parameters` are compared, against the
  // values the Dataset was built with (reference Booster::CheckDatasetResetConfig)
  auto o = Config::Str2Map(old_parameters), n = Config::Str2Map(new_parameters);
  Config::KeyAliasTransform(&o);
  Config::KeyAliasTransform(&n);
  static const char* kDatasetParams[] = {"max_bin", "max_bin_by_feature", "bin_construct_sample_cnt", "min_data_in_bin",
                                         "use_missing", "zero_as_missing", "categorical_feature", "feature_pre_filter",
                                         "enable_bundle", "data_random_seed", "is_enable_sparse", "header",
                                         "two_round", "label_column", "weight_column", "group_column",
                                         "ignore_column", "linear_tree", "precise_float_parser"};
  // typed comparison of the dataset keys only (the other parameters may legitimately change)
  ParamMap ob, nb;
  for (const char* k : kDatasetParams) {
    if (o.count(k)) ob[k] = o[k];
  }
  nb = ob;
  for (const char* k : kDatasetParams) {
    if (n.count(k)) nb[k] = n[k];
  }
  Config before, after;
  before.Set(ob);
  after.Set(nb);
  auto lines = [](const std::string& dump) {
    std::unordered_map<std::string, std::string> m;
    for (auto& l : common::SplitLines(dump.c_str())) {
      const size_t c = l.find(": ");
      if (l.size() > 3 && l.front() == '[' && c != std::string::npos) m[l.substr(1, c - 1)] = l.substr(c + 2);
    }
    return m;
  };
  auto bm = lines(before.ToString()), am = lines(after.ToString());
  if (n.count("forcedbins_filename")) Log::Fatal("Cannot change forced bins after constructed Dataset handle.");
  for (const char* k : kDatasetParams) {
    if (!n.count(k)) continue;
    if (bm[k] != am[k]) Log::Fatal("Cannot change %s after constructed Dataset handle.", k);
  }
  if (n.count("pre_partition") && (o.count("pre_partition") ? o["pre_partition"] : "false") != n["pre_partition"]) {
    Config a, b;
    a.Set({{"pre_partition", o.count("pre_partition") ? o["pre_partition"] : "false"}});
    b.Set({{"pre_partition", n["pre_partition"]}});
    if (a.pre_partition != b.pre_partition) Log::Fatal("Cannot change pre_partition after constructed Dataset handle.");
  }
  if (n.count("min_data_in_leaf")) {
    Config a, b;
    ParamMap ao;
    for (const char* k : {"min_data_in_leaf", "feature_pre_filter"}) {
      if (o.count(k)) ao[k] = o[k];
    }
    a.Set(ao);
    b.Set({{"min_data_in_leaf", n["min_data_in_leaf"]}});
    if (b.min_data_in_leaf < a.min_data_in_leaf && a.feature_pre_filter) {
      Log::Fatal("Reducing `min_data_in_leaf` with `feature_pre_filter=true` may cause unexpected behaviour for "
                 "features that were pre-filtered by the larger `min_data_in_leaf`.\nYou need to set "
                 "`feature_pre_filter=false` to dynamically change the `min_data_in_leaf`.");
    }
  }
  API_END();
}

int LGBM_DatasetGetNumData(DatasetHandle handle, int* out) {
  API_BEGIN();
  *out = D(handle)->ds->num_data();
  API_END();
}

int LGBM_DatasetGetNumFeature(DatasetHandle handle, int* out) {
  API_BEGIN();
  *out = D(handle)->ds->num_total_features();
  API_END();
}

int LGBM_DatasetGetFeatureNumBin(DatasetHandle handle, int feature, int* out) {
  API_BEGIN();
  const Dataset* ds = D(handle)->ds.get();
  if (feature < 0 || feature >= ds->num_total_features()) Log::Fatal("Tried to retrieve number of bins for feature index %d", feature);
  int inner = ds->InnerIndex(feature);
  *out = inner < 0 ? 0 : ds->feature(inner).num_bin;
  API_END();
}

int LGBM_DatasetAddFeaturesFrom(DatasetHandle target, DatasetHandle source) {
  API_BEGIN();
  D(target)->ds->AddFeaturesFrom(*D(source)->ds);
  API_END();
}

// ---------------------------------------------------------------------------
int LGBM_BoosterCreate(const DatasetHandle train_data, const char* parameters, BoosterHandle* out) {
  API_BEGIN();
  *out = new Booster(D(train_data), parameters);
  API_END();
}

int LGBM_BoosterCreateFromModelfile(const char* filename, int* out_num_iterations, BoosterHandle* out) {
  API_BEGIN();
  std::ifstream in(filename, std::ios::binary);
  if (!in) Log::Fatal("Model file %s is not available", filename);
  std::string s((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  auto* b = new Booster(s.data(), s.size());
  *out_num_iterations = b->boosting_->GetCurrentIteration();
  *out = b;
  API_END();
}

int LGBM_BoosterLoadModelFromString(const char* model_str, int* out_num_iterations, BoosterHandle* out) {
  API_BEGIN();
  auto* b = new Booster(model_str, std::strlen(model_str));
  *out_num_iterations = b->boosting_->GetCurrentIteration();
  *out = b;
  API_END();
}

namespace {
std::string JsonQuote(const std::string& v) {
  std::string o = "\"";
  for (char ch : v) {
    if (ch == '"' || ch == '\\') o += '\\';
    o += ch;
  }
  return o + "\"";
}

bool AllInts(const std::vector<std::string>& parts) {
  for (auto& t : parts) {
    if (t.empty() || t.find_first_not_of("-0123456789") != std::string::npos) return false;
  }
  return !parts.empty();
}
}  // namespace

// The model's "parameters:" section as a typed JSON object (reference GBDT::GetLoadedParam,
// gbdt.h): values typed by the parameter table, empty values skipped, unknown keys warned
// about and dropped.
int LGBM_BoosterGetLoadedParam(BoosterHandle handle, int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  std::string p = B(handle)->boosting_->loaded_parameter();
  std::stringstream ss;
  ss << "{";
  bool first = true;
  for (auto& line : common::SplitLines(p.c_str())) {
    if (line.size() < 4 || line.front() != '[' || line.back() != ']') continue;
    size_t c = line.find(": ");
    if (c == std::string::npos) continue;
    const std::string k = line.substr(1, c - 1), v = line.substr(c + 2, line.size() - c - 3);
    if (v.empty()) continue;
    const std::string kind = Config::ParameterKind(k);
    if (kind.empty()) {
      Log::Warning("Ignoring unrecognized parameter '%s' found in model string.", k.c_str());
      continue;
    }
    std::string js;
    const auto parts = common::Split(v, ',');
    if (k == "interaction_constraints") {
      js = "[" + v + "]";
    } else if (k == "categorical_feature" && AllInts(parts)) {
      js = "[" + v + "]";
    } else if (kind == "STR") {
      js = JsonQuote(v);
    } else if (kind == "BOOL") {
      js = (v == "1" || v == "true") ? "true" : "false";
    } else if (kind == "INT" || kind == "DBL") {
      js = v;
    } else if (kind == "VSTR") {
      js = "[";
      for (size_t i = 0; i < parts.size(); ++i) js += (i ? "," : "") + JsonQuote(parts[i]);
      js += "]";
    } else {
      js = "[" + v + "]";
    }
    ss << (first ? "" : ", ") << JsonQuote(k) << ": " << js;
    first = false;
  }
  ss << "}";
  CopyStr(ss.str(), buffer_len, out_len, out_str);
  API_END();
}

int LGBM_BoosterFree(BoosterHandle handle) {
  API_BEGIN();
  delete B(handle);
  API_END();
}

int LGBM_BoosterShuffleModels(BoosterHandle handle, int start_iter, int end_iter) {
  API_BEGIN();
  std::unique_lock<std::shared_mutex> lk(B(handle)->mu_);
  B(handle)->boosting_->ShuffleModels(start_iter, end_iter);
  API_END();
}

int LGBM_BoosterMerge(BoosterHandle handle, BoosterHandle other_handle) {
  API_BEGIN();
  std::unique_lock<std::shared_mutex> lk(B(handle)->mu_);
  B(handle)->boosting_->MergeFrom(B(other_handle)->boosting_.get());
  API_END();
}

int LGBM_BoosterAddValidData(BoosterHandle handle, const DatasetHandle valid_data) {
  API_BEGIN();
  B(handle)->AddValidData(D(valid_data));
  API_END();
}

int LGBM_BoosterResetTrainingData(BoosterHandle handle, const DatasetHandle train_data) {
  API_BEGIN();
  Booster* b = B(handle);
  std::unique_lock<std::shared_mutex> lk(b->mu_);
  b->train_ = D(train_data);
  b->CreateObjectiveAndMetrics();
  b->boosting_->ResetTrainingData(b->train_->ds.get(), b->objective_.get(), Booster::MetricPtrs(b->train_metrics_));
  API_END();
}

int LGBM_BoosterResetParameter(BoosterHandle handle, const char* parameters) {
  API_BEGIN();
  B(handle)->ResetParameter(parameters);
  API_END();
}

int LGBM_BoosterGetNumClasses(BoosterHandle handle, int* out_len) {
  API_BEGIN();
  *out_len = B(handle)->boosting_->NumberOfClasses();
  API_END();
}

int LGBM_BoosterGetLinear(BoosterHandle handle, int* out) {
  API_BEGIN();
  *out = B(handle)->boosting_->NumberOfTotalModel() > 0 && B(handle)->boosting_->GetTree(0)->is_linear();
  API_END();
}

int LGBM_BoosterUpdateOneIter(BoosterHandle handle, int* is_finished) {
  API_BEGIN();
  *is_finished = B(handle)->TrainOneIter() ? 1 : 0;
  API_END();
}

int LGBM_BoosterRefit(BoosterHandle handle, const int32_t* leaf_preds, int32_t nrow, int32_t ncol) {
  API_BEGIN();
  std::unique_lock<std::shared_mutex> lk(B(handle)->mu_);
  std::vector<std::vector<int>> lp(nrow, std::vector<int>(ncol));
  for (int i = 0; i < nrow; ++i)
    for (int j = 0; j < ncol; ++j) lp[i][j] = leaf_preds[static_cast<size_t>(i) * ncol + j];
  B(handle)->boosting_->RefitTree(lp);
  API_END();
}

int LGBM_BoosterUpdateOneIterCustom(BoosterHandle handle, const float* grad, const float* hess, int* is_finished) {
  API_BEGIN();
  *is_finished = B(handle)->TrainOneIterCustom(grad, hess) ? 1 : 0;
  API_END();
}

int LGBM_BoosterRollbackOneIter(BoosterHandle handle) {
  API_BEGIN();
  std::unique_lock<std::shared_mutex> lk(B(handle)->mu_);
  B(handle)->boosting_->RollbackOneIter();
  API_END();
}

int LGBM_BoosterGetCurrentIteration(BoosterHandle handle, int* out_iteration) {
  API_BEGIN();
  *out_iteration = B(handle)->boosting_->GetCurrentIteration();
  API_END();
}

int LGBM_BoosterNumModelPerIteration(BoosterHandle handle, int* out) {
  API_BEGIN();
  *out = B(handle)->boosting_->NumModelPerIteration();
  API_END();
}

int LGBM_BoosterNumberOfTotalModel(BoosterHandle handle, int* out_models) {
  API_BEGIN();
  *out_models = B(handle)->boosting_->NumberOfTotalModel();
  API_END();
}

int LGBM_BoosterGetEvalCounts(BoosterHandle handle, int* out_len) {
  API_BEGIN();
  *out_len = static_cast<int>(B(handle)->boosting_->GetEvalNames().size());
  API_END();
}

int LGBM_BoosterGetEvalNames(BoosterHandle handle, const int len, int* out_len, const size_t buffer_len,
                             size_t* out_buffer_len, char** out_strs) {
  API_BEGIN();
  CopyStrings(B(handle)->boosting_->GetEvalNames(), len, out_len, buffer_len, out_buffer_len, out_strs);
  API_END();
}

int LGBM_BoosterGetFeatureNames(BoosterHandle handle, const int len, int* out_len, const size_t buffer_len,
                                size_t* out_buffer_len, char** out_strs) {
  API_BEGIN();
  CopyStrings(B(handle)->boosting_->FeatureNames(), len, out_len, buffer_len, out_buffer_len, out_strs);
  API_END();
}

int LGBM_BoosterValidateFeatureNames(BoosterHandle handle, const char** data_names, int data_num_features) {
  API_BEGIN();
  const auto& names = B(handle)->boosting_->FeatureNames();
  if (static_cast<int>(names.size()) != data_num_features) {
    Log::Fatal("Model was trained on %d features, but got %d input features to predict.",
               static_cast<int>(names.size()), data_num_features);
  }
  for (int i = 0; i < data_num_features; ++i) {
    if (names[i] != data_names[i]) {
      Log::Fatal("Expected '%s' at position %d but found '%s'", names[i].c_str(), i, data_names[i]);
    }
  }
  API_END();
}

int LGBM_BoosterGetNumFeature(BoosterHandle handle, int* out_len) {
  API_BEGIN();
  *out_len = B(handle)->boosting_->MaxFeatureIdx() + 1;
  API_END();
}

int LGBM_BoosterGetEval(BoosterHandle handle, int data_idx, int* out_len, double* out_results) {
  API_BEGIN();
  std::unique_lock<std::shared_mutex> lk(B(handle)->mu_);
  auto r = B(handle)->boosting_->GetEvalAt(data_idx);
  *out_len = static_cast<int>(r.size());
  std::copy(r.begin(), r.end(), out_results);
  API_END();
}

int LGBM_BoosterGetNumPredict(BoosterHandle handle, int data_idx, int64_t* out_len) {
  API_BEGIN();
  *out_len = B(handle)->boosting_->GetNumPredictAt(data_idx);
  API_END();
}

int LGBM_BoosterGetPredict(BoosterHandle handle, int data_idx, int64_t* out_len, double* out_result) {
  API_BEGIN();
  std::unique_lock<std::shared_mutex> lk(B(handle)->mu_);
  B(handle)->boosting_->GetPredictAt(data_idx, out_result, out_len);
  API_END();
}

int LGBM_BoosterPredictForFile(BoosterHandle handle, const char* data_filename, int data_has_header, int predict_type,
                               int start_iteration, int num_iteration, const char* parameter,
                               const char* result_filename) {
  API_BEGIN();
  Booster* b = B(handle);
  OwnedSparseSource rows;
  std::vector<float> labels;
  int label_idx = 0;
  Config pc = ParseConfig(parameter);
  if (!pc.label_column.empty() && !common::StartsWith(pc.label_column, "name:")) label_idx = common::AtoiOrDie(pc.label_column);
  const int nf = b->boosting_->MaxFeatureIdx() + 1;
  const std::string& parser_cfg = b->boosting_->parser_config();
  if (!parser_cfg.empty()) {
    // the model was trained on rows of a custom parser: predict through the same class
    auto parser = CreateCustomParser(parser_cfg);
    std::ifstream in(data_filename);
    if (!in) Log::Fatal("Data file %s doesn't exist.", data_filename);
    std::string line;
    if (data_has_header) std::getline(in, line);
    int data_nf = 0;
    while (std::getline(in, line)) {
      if (!line.empty() && line.back() == '\r') line.pop_back();
      rows.rows.emplace_back();
      double lab = 0.0;
      parser->ParseOneLine(line.c_str(), &rows.rows.back(), &lab);
      labels.push_back(static_cast<float>(lab));
      // a negative index is a parser bug; an index past the model's features (a column the
      // training data never had) is an error unless predict_disable_shape_check is set, and is
      // then dropped, as the reference's CopyToPredictBuffer (predictor.hpp:259) ignores it
      auto& r = rows.rows.back();
      for (const auto& kv : r) {
        if (kv.first < 0) Log::Fatal("The custom parser produced feature index %d", kv.first);
        data_nf = std::max(data_nf, kv.first + 1);
      }
      if (data_nf > nf && !pc.predict_disable_shape_check) {
        // (reference predictor.hpp:176-178)
        Log::Fatal("The number of features in data (%d) is not the same as it was in training data (%d).\n"
                   "You can set ``predict_disable_shape_check=true`` to discard this error, but please be aware "
                   "what you are doing.", data_nf, nf);
      }
      r.erase(std::remove_if(r.begin(), r.end(), [nf](const auto& kv) { return kv.first >= nf; }),
              r.end());
    }
    rows.ncol = nf;
  } else {
    ParseTextFile(data_filename, data_has_header != 0, label_idx, &rows, &labels, nullptr, nullptr, {}, -1, nullptr, -1,
                  nullptr);
  }
  // a file without the label column has one fewer column than the model: shift back in that case
  if (parser_cfg.empty() && rows.ncol == nf - 1 && label_idx == 0) {
    for (auto& r : rows.rows) {
      for (auto& kv : r) kv.first += 1;
    }
    // first value was consumed as label: put it back as feature 0
    for (size_t i = 0; i < rows.rows.size(); ++i) rows.rows[i].insert(rows.rows[i].begin(), {0, labels[i]});
    rows.ncol = nf;
  }
  rows.ncol = std::max(rows.ncol, nf);
  std::string params = parameter ? parameter : "";
  params += " predict_disable_shape_check=true";
  const int per = b->boosting_->NumPredictOneRow(start_iteration, num_iteration, predict_type == C_API_PREDICT_LEAF_INDEX,
                                                 predict_type == C_API_PREDICT_CONTRIB);
  std::vector<double> out(rows.rows.size() * static_cast<size_t>(per));
  int64_t len;
  PredictRows(b, rows, predict_type, start_iteration, num_iteration, params.c_str(), &len, out.data());
  std::ofstream fo(result_filename);
  for (size_t i = 0; i < rows.rows.size(); ++i) {
    for (int k = 0; k < per; ++k) {
      if (k) fo << '\t';
      fo << common::Format17(out[i * per + k]);
    }
    fo << '\n';
  }
  API_END();
}

int LGBM_BoosterCalcNumPredict(BoosterHandle handle, int num_row, int predict_type, int start_iteration,
                               int num_iteration, int64_t* out_len) {
  API_BEGIN();
  *out_len = static_cast<int64_t>(num_row) *
             B(handle)->boosting_->NumPredictOneRow(start_iteration, num_iteration,
                                                    predict_type == C_API_PREDICT_LEAF_INDEX,
                                                    predict_type == C_API_PREDICT_CONTRIB);
  API_END();
}

int LGBM_BoosterPredictForCSR(BoosterHandle handle, const void* indptr, int indptr_type, const int32_t* indices,
                              const void* data, int data_type, int64_t nindptr, int64_t nelem, int64_t num_col,
                              int predict_type, int start_iteration, int num_iteration, const char* parameter,
                              int64_t* out_len, double* out_result) {
  API_BEGIN();
  CSRSource src(indptr, indptr_type == C_API_DTYPE_INT64, indices, data, data_type == C_API_DTYPE_FLOAT64, nindptr,
                nelem, num_col);
  PredictRows(B(handle), src, predict_type, start_iteration, num_iteration, parameter, out_len, out_result);
  API_END();
}

int LGBM_BoosterPredictForCSRSingleRow(BoosterHandle handle, const void* indptr, int indptr_type,
                                       const int32_t* indices, const void* data, int data_type, int64_t nindptr,
                                       int64_t nelem, int64_t num_col, int predict_type, int start_iteration,
                                       int num_iteration, const char* parameter, int64_t* out_len,
                                       double* out_result) {
  return LGBM_BoosterPredictForCSR(handle, indptr, indptr_type, indices, data, data_type, nindptr, nelem, num_col,
                                   predict_type, start_iteration, num_iteration, parameter, out_len, out_result);
}

int LGBM_BoosterPredictForCSC(BoosterHandle handle, const void* col_ptr, int col_ptr_type, const int32_t* indices,
                              const void* data, int data_type, int64_t ncol_ptr, int64_t nelem, int64_t num_row,
                              int predict_type, int start_iteration, int num_iteration, const char* parameter,
                              int64_t* out_len, double* out_result) {
  API_BEGIN();
  (void)nelem;
  auto src = CSCToRows(col_ptr, col_ptr_type, indices, data, data_type, ncol_ptr, num_row);
  PredictRows(B(handle), *src, predict_type, start_iteration, num_iteration, parameter, out_len, out_result);
  API_END();
}

int LGBM_BoosterPredictForMat(BoosterHandle handle, const void* data, int data_type, int32_t nrow, int32_t ncol,
                              int is_row_major, int predict_type, int start_iteration, int num_iteration,
                              const char* parameter, int64_t* out_len, double* out_result) {
  API_BEGIN();
  DenseSource src(data, data_type == C_API_DTYPE_FLOAT64, nrow, ncol, is_row_major != 0);
  PredictRows(B(handle), src, predict_type, start_iteration, num_iteration, parameter, out_len, out_result);
  API_END();
}

int LGBM_BoosterPredictForMatSingleRow(BoosterHandle handle, const void* data, int data_type, int ncol,
                                       int is_row_major, int predict_type, int start_iteration, int num_iteration,
                                       const char* parameter, int64_t* out_len, double* out_result) {
  return LGBM_BoosterPredictForMat(handle, data, data_type, 1, ncol, is_row_major, predict_type, start_iteration,
                                   num_iteration, parameter, out_len, out_result);
}

int LGBM_BoosterPredictForMats(BoosterHandle handle, const void** data, int data_type, int32_t nrow, int32_t ncol,
                               int predict_type, int start_iteration, int num_iteration, const char* parameter,
                               int64_t* out_len, double* out_result) {
  API_BEGIN();
  std::vector<DenseSource> mats;
  for (int i = 0; i < nrow; ++i) mats.emplace_back(data[i], data_type == C_API_DTYPE_FLOAT64, 1, ncol, true);
  MultiDenseSource src(std::move(mats));
  PredictRows(B(handle), src, predict_type, start_iteration, num_iteration, parameter, out_len, out_result);
  API_END();
}

int LGBM_BoosterSaveModel(BoosterHandle handle, int start_iteration, int num_iteration, int feature_importance_type,
                          const char* filename) {
  API_BEGIN();
  std::shared_lock<std::shared_mutex> lk(B(handle)->mu_);
  B(handle)->boosting_->SaveModelToFile(start_iteration, num_iteration, feature_importance_type, filename);
  API_END();
}

int LGBM_BoosterSaveModelToString(BoosterHandle handle, int start_iteration, int num_iteration,
                                  int feature_importance_type, int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  std::shared_lock<std::shared_mutex> lk(B(handle)->mu_);
  CopyStr(B(handle)->boosting_->SaveModelToString(start_iteration, num_iteration, feature_importance_type), buffer_len,
          out_len, out_str);
  API_END();
}

int LGBM_BoosterDumpModel(BoosterHandle handle, int start_iteration, int num_iteration, int feature_importance_type,
                          int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  std::shared_lock<std::shared_mutex> lk(B(handle)->mu_);
  CopyStr(B(handle)->boosting_->DumpModel(start_iteration, num_iteration, feature_importance_type), buffer_len,
          out_len, out_str);
  API_END();
}

int LGBM_BoosterConvertModelToIfElse(BoosterHandle handle, int num_iteration, int64_t buffer_len, int64_t* out_len,
                                     char* out_str) {
  API_BEGIN();
  CopyStr(B(handle)->boosting_->ModelToIfElse(num_iteration), buffer_len, out_len, out_str);
  API_END();
}

int LGBM_BoosterGetLeafValue(BoosterHandle handle, int tree_idx, int leaf_idx, double* out_val) {
  API_BEGIN();
  *out_val = B(handle)->boosting_->GetLeafValue(tree_idx, leaf_idx);
  API_END();
}

int LGBM_BoosterSetLeafValue(BoosterHandle handle, int tree_idx, int leaf_idx, double val) {
  API_BEGIN();
  std::unique_lock<std::shared_mutex> lk(B(handle)->mu_);
  B(handle)->boosting_->SetLeafValue(tree_idx, leaf_idx, val);
  API_END();
}

int LGBM_BoosterFeatureImportance(BoosterHandle handle, int num_iteration, int importance_type, double* out_results) {
  API_BEGIN();
  auto imp = B(handle)->boosting_->FeatureImportance(num_iteration, importance_type);
  std::copy(imp.begin(), imp.end(), out_results);
  API_END();
}

int LGBM_BoosterGetUpperBoundValue(BoosterHandle handle, double* out_results) {
  API_BEGIN();
  GBDT* g = B(handle)->boosting_.get();
  double s = 0.0;
  for (int i = 0; i < g->NumberOfTotalModel(); ++i) {
    const Tree* t = g->GetTree(i);
    double m = t->LeafOutput(0);
    for (int l = 1; l < t->num_leaves(); ++l) m = std::max(m, t->LeafOutput(l));
    s += m;
  }
  *out_results = s;
  API_END();
}

int LGBM_BoosterGetLowerBoundValue(BoosterHandle handle, double* out_results) {
  API_BEGIN();
  GBDT* g = B(handle)->boosting_.get();
  double s = 0.0;
  for (int i = 0; i < g->NumberOfTotalModel(); ++i) {
    const Tree* t = g->GetTree(i);
    double m = t->LeafOutput(0);
    for (int l = 1; l < t->num_leaves(); ++l) m = std::min(m, t->LeafOutput(l));
    s += m;
  }
  *out_results = s;
  API_END();
}

int LGBM_BoosterGetDeviceName(BoosterHandle handle, int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  TreeLearner* l = B(handle)->boosting_->tree_learner();
  CopyStr(l ? l->DeviceName() : "none", buffer_len, out_len, out_str);
  API_END();
}

// ---------------------------------------------------------------------------
int LGBM_NetworkInit(const char* machines, int local_listen_port, int listen_time_out, int num_machines) {
  API_BEGIN();
  Config c;
  c.machines = machines;
  c.local_listen_port = local_listen_port;
  c.time_out = listen_time_out;
  c.num_machines = num_machines;
  if (num_machines > 1) Network::Init(c);
  API_END();
}

int LGBM_NetworkFree() {
  API_BEGIN();
  Network::Dispose();
  API_END();
}

int LGBM_NetworkInitWithFunctions(int num_machines, int rank, void* reduce_scatter_ext_fun, void* allgather_ext_fun) {
  API_BEGIN();
  if (num_machines > 1) {
    using RSRaw = void (*)(char*, comm_size_t, int, const comm_size_t*, const comm_size_t*, int, char*, comm_size_t,
                           const ReduceFunction&);
    using AGRaw = void (*)(char*, comm_size_t, const comm_size_t*, const comm_size_t*, int, char*, comm_size_t);
    if (allgather_ext_fun == nullptr) Log::Fatal("LGBM_NetworkInitWithFunctions needs an allgather function");
    auto ag = reinterpret_cast<AGRaw>(allgather_ext_fun);
    // a null reduce-scatter (e.g. a Python / torch.distributed allgather-only transport) is
    // served by allgather + local reduction inside Network
    ReduceScatterFunction rs = nullptr;
    if (reduce_scatter_ext_fun != nullptr) rs = reinterpret_cast<RSRaw>(reduce_scatter_ext_fun);
    Network::Init(num_machines, rank, rs, AllgatherFunction(ag));
  }
  API_END();
}

int LGBM_SetMaxThreads(int num_threads) {
  API_BEGIN();
  SetMaxNumThreads(num_threads);
  API_END();
}

int LGBM_GetMaxThreads(int* out) {
  API_BEGIN();
  *out = MaxNumThreadsSetting();
  API_END();
}

// OpenMP team size a parallel region entered from the calling thread would use (diagnostic:
// the effective num_threads / LGBM_SetMaxThreads setting as applied on this thread)
int LGBM_GetEffectiveThreads(int* out) {
  API_BEGIN();
  *out = omp_get_max_threads();
  API_END();
}

int LGBM_PhaseTimerReport(int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  CopyStr(PhaseTimer::Global().Report(), buffer_len, out_len, out_str);
  API_END();
}

int LGBM_DeviceCount(int* out) {
  API_BEGIN();
  *out = device::DeviceCount();
  API_END();
}

int LGBM_BoosterGetGradients(BoosterHandle handle, int64_t* out_len, float* grad, float* hess) {
  API_BEGIN();
  std::vector<score_t> g, h;
  B(handle)->boosting_->GetGradients(&g, &h);
  *out_len = static_cast<int64_t>(g.size());
  if (grad) std::copy(g.begin(), g.end(), grad);
  if (hess) std::copy(h.begin(), h.end(), hess);
  API_END();
}

int LGBM_DatasetGetGroupLayout(DatasetHandle handle, int* num_groups, int* num_total_bin, int* bin_width,
                               int32_t* hist_start) {
  API_BEGIN();
  const Dataset* d = D(handle)->ds.get();
  *num_groups = d->num_groups();
  *num_total_bin = d->num_total_bin();
  *bin_width = d->bin_width();
  if (hist_start) {
    for (int g = 0; g < d->num_groups(); ++g) hist_start[g] = d->group(g).hist_start;
  }
  API_END();
}

int LGBM_DatasetGetGroupBins(DatasetHandle handle, uint16_t* out) {
  API_BEGIN();
  const Dataset* d = D(handle)->ds.get();
  const int ng = d->num_groups();
#pragma omp parallel for schedule(static)
  for (data_size_t i = 0; i < d->num_data(); ++i) {
    for (int g = 0; g < ng; ++g) out[static_cast<size_t>(i) * ng + g] = static_cast<uint16_t>(d->GroupBin(i, g));
  }
  API_END();
}

int LGBM_DeviceHistogram(DatasetHandle handle, const float* grad, const float* hess, const int32_t* rows,
                         int32_t num_rows, double* out_hist) {
  API_BEGIN();
  device::DeviceHistogram(D(handle)->ds.get(), grad, hess, rows, num_rows, out_hist);
  API_END();
}

// Direct frontier-kernel tests (device_api.h TestFrontierHist / TestFrontierPartition): a device
// learner with `parameters` on the Dataset, one k_f_hist / k_f_partition launch over row subsets.
int LGBM_DeviceTestFrontierHist(DatasetHandle handle, const char* parameters, const float* grad, const float* hess,
                                const int32_t* rows, const int32_t* offsets, int k, double* out, uint16_t* levels) {
  API_BEGIN();
  Config cfg = ParseConfig(parameters);
  cfg.device_type = "gpu";
  device::TestFrontierHist(D(handle)->ds.get(), cfg, grad, hess, rows, offsets, k, out, levels);
  API_END();
}

int LGBM_DeviceTestFrontierScan(DatasetHandle handle, const char* parameters, const float* grad, const float* hess,
                                double* out, double* ref) {
  API_BEGIN();
  Config cfg = ParseConfig(parameters);
  cfg.device_type = "gpu";
  device::TestFrontierScan(D(handle)->ds.get(), cfg, grad, hess, out, ref);
  API_END();
}

int LGBM_DeviceTestFrontierPartition(DatasetHandle handle, const char* parameters, const int32_t* rows,
                                     const int32_t* offsets, int k, const int32_t* feats, const int32_t* thr,
                                     const int32_t* dleft, const uint32_t* catbits, int32_t* out_rows,
                                     int32_t* out_left, int32_t* exp_rows, int32_t* exp_left) {
  API_BEGIN();
  Config cfg = ParseConfig(parameters);
  cfg.device_type = "gpu";
  device::TestFrontierPartition(D(handle)->ds.get(), cfg, rows, offsets, k, feats, thr, dleft, catbits, out_rows,
                                out_left, exp_rows, exp_left);
  API_END();
}

int LGBM_DeviceSampleRows(int mode, int32_t num_rows, int num_class, float* grad, float* hess, const float* label,
                          double fraction, double pos_fraction, double neg_fraction, double top_rate,
                          double other_rate, int bagging_seed, uint32_t goss_seed, int rounds, int32_t* out_rows,
                          int32_t* out_count) {
  API_BEGIN();
  *out_count = device::SampleRowsOnDevice(mode, num_rows, num_class, grad, hess, label, fraction, pos_fraction,
                                          neg_fraction, top_rate, other_rate, bagging_seed, goss_seed, rounds,
                                          out_rows);
  API_END();
}

int LGBM_DeviceSynchronize() {
  API_BEGIN();
  device::DeviceSynchronize();
  API_END();
}

int LGBM_DeviceCommGetUniqueId(char* out, int64_t buffer_len, int64_t* out_len) {
  API_BEGIN();
  std::string id = device::CommGetUniqueId();
  *out_len = static_cast<int64_t>(id.size());
  if (out != nullptr && buffer_len >= *out_len) std::memcpy(out, id.data(), id.size());
  API_END();
}

int LGBM_DeviceCommInit(const char* unique_id, int64_t id_len, int num_ranks, int rank, int device_id) {
  API_BEGIN();
  device::CommInit(std::string(unique_id, unique_id + id_len), num_ranks, rank, device_id);
  API_END();
}

int LGBM_DeviceCommFree() {
  API_BEGIN();
  device::CommFree();
  API_END();
}

// ============================================================================
// Arrow, streaming / sampled constructors, serialized references, fast
// single-row and sparse-output prediction (reference src/c_api.cpp:1245-2960).
namespace {

class FuncSource : public RowSource {
 public:
  using RowFn = std::function<void(int idx, std::vector<std::pair<int, double>>& row)>;
  FuncSource(RowFn* fn, int nrow, int ncol) : fn_(fn), nrow_(nrow), ncol_(ncol) {}
  data_size_t num_rows() const override { return nrow_; }
  int num_cols() const override { return ncol_; }
  void GetRow(data_size_t i, std::vector<std::pair<int, double>>* out) const override {
    out->clear();
    (*fn_)(static_cast<int>(i), *out);
  }

 private:
  RowFn* fn_;
  int nrow_, ncol_;
};

struct FastConfig {
  Booster* booster;
  int predict_type, start_iteration, num_iteration, data_type;
  int64_t ncol;
  Config config;
  std::unique_ptr<PredictionEarlyStop> es;
};

// One row through the booster without OpenMP or config parsing.
void PredictOneRow(FastConfig* fc, const std::vector<std::pair<int, double>>& row, int64_t* out_len, double* out) {
  Booster* b = fc->booster;
  std::shared_lock<std::shared_mutex> lk(b->mu_);
  GBDT* g = b->boosting_.get();
  const bool leaf = fc->predict_type == C_API_PREDICT_LEAF_INDEX;
  const bool contrib = fc->predict_type == C_API_PREDICT_CONTRIB;
  g->InitPredict(fc->start_iteration, fc->num_iteration, contrib);
  const int nf = std::max<int64_t>(g->MaxFeatureIdx() + 1, fc->ncol);
  thread_local std::vector<double> x;
  x.assign(nf, 0.0);
  for (auto& kv : row) if (kv.first < nf) x[kv.first] = kv.second;
  if (leaf) g->PredictLeafIndex(x.data(), out);
  else if (contrib) g->PredictContrib(x.data(), out);
  else if (fc->predict_type == C_API_PREDICT_RAW_SCORE) g->PredictRaw(x.data(), out, fc->es.get());
  else g->Predict(x.data(), out, fc->es.get());
  *out_len = g->NumPredictOneRow(fc->start_iteration, fc->num_iteration, leaf, contrib);
}

FastConfig* MakeFast(BoosterHandle handle, int predict_type, int start_iteration, int num_iteration, int data_type,
                     int64_t ncol, const char* parameter) {
  auto fc = std::make_unique<FastConfig>();
  fc->booster = B(handle);
  fc->predict_type = predict_type;
  fc->start_iteration = start_iteration;
  fc->num_iteration = num_iteration;
  fc->data_type = data_type;
  fc->ncol = ncol;
  fc->config = ParseConfig(parameter);
  std::string es_type = "none";
  const GBDT* g = fc->booster->boosting_.get();
  if (fc->config.pred_early_stop && predict_type != C_API_PREDICT_LEAF_INDEX && predict_type != C_API_PREDICT_CONTRIB &&
      !g->NeedAccuratePrediction()) {
    es_type = g->NumberOfClasses() == 1 ? "binary" : "multiclass";
  }
  fc->es = std::make_unique<PredictionEarlyStop>(es_type, fc->config.pred_early_stop_freq,
                                                 fc->config.pred_early_stop_margin);
  return fc.release();
}

struct ByteBuffer {
  std::vector<char> data;
};

}  // namespace

void LGBM_SetLastError(const char* msg) { SetLastError(msg); }

int LGBM_DatasetCreateFromArrow(int64_t n_chunks, const struct ArrowArray* chunks, const struct ArrowSchema* schema,
                                const char* parameters, const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  ArrowTable table(n_chunks, chunks, schema);
  ArrowSource src(table);
  *out = BuildFromSource(src, parameters, reference);
  D(*out)->ds->set_feature_names(table.names());
  API_END();
}

int LGBM_DatasetSetFieldFromArrow(DatasetHandle handle, const char* field_name, int64_t n_chunks,
                                  const struct ArrowArray* chunks, const struct ArrowSchema* schema) {
  API_BEGIN();
  ArrowTable table(n_chunks, chunks, schema);
  const std::string name(field_name);
  // a multi-column table is accepted for init_score only: one column per class, which is
  // the class-major layout the field stores
  if (table.num_columns() != 1 && !(name == "init_score" && table.num_columns() > 1)) {
    Log::Fatal("Arrow field %s must have exactly one column", field_name);
  }
  std::vector<double> v;
  for (int c = 0; c < table.num_columns(); ++c) {
    const std::vector<double> col = table.Column(c);
    v.insert(v.end(), col.begin(), col.end());
  }
  if (name == "group" || name == "query" || name == "position") {
    std::vector<int32_t> iv(v.begin(), v.end());
    if (LGBM_DatasetSetField(handle, field_name, iv.data(), static_cast<int>(iv.size()), C_API_DTYPE_INT32) != 0) {
      throw std::runtime_error(LGBM_GetLastError());
    }
  } else if (LGBM_DatasetSetField(handle, field_name, v.data(), static_cast<int>(v.size()), C_API_DTYPE_FLOAT64) != 0) {
    throw std::runtime_error(LGBM_GetLastError());
  }
  API_END();
}

int LGBM_BoosterPredictForArrow(BoosterHandle handle, int64_t n_chunks, const struct ArrowArray* chunks,
                                const struct ArrowSchema* schema, int predict_type, int start_iteration,
                                int num_iteration, const char* parameter, int64_t* out_len, double* out_result) {
  API_BEGIN();
  ArrowTable table(n_chunks, chunks, schema);
  ArrowSource src(table);
  PredictRows(B(handle), src, predict_type, start_iteration, num_iteration, parameter, out_len, out_result);
  API_END();
}

int LGBM_DatasetCreateFromCSRFunc(void* get_row_funptr, int num_rows, int64_t num_col, const char* parameters,
                                  const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  FuncSource src(static_cast<FuncSource::RowFn*>(get_row_funptr), num_rows, static_cast<int>(num_col));
  *out = BuildFromSource(src, parameters, reference);
  API_END();
}

int LGBM_DatasetCreateFromSampledColumn(double** sample_data, int** sample_indices, int32_t ncol,
                                        const int* num_per_col, int32_t num_sample_row, int32_t num_local_row,
                                        int64_t num_dist_row, const char* parameters, DatasetHandle* out) {
  API_BEGIN();
  (void)num_dist_row;
  // bin boundaries come from the sampled non-zero values; rows arrive later via PushRows
  OwnedSparseSource sample;
  sample.ncol = ncol;
  sample.rows.resize(num_sample_row);
  for (int32_t c = 0; c < ncol; ++c) {
    for (int k = 0; k < num_per_col[c]; ++k) {
      const int r = sample_indices[c][k];
      if (r >= 0 && r < num_sample_row) sample.rows[r].emplace_back(c, sample_data[c][k]);
    }
  }
  Config cfg = ParseConfig(parameters);
  Dataset ref;
  ref.Construct(sample, cfg, nullptr, {}, CategoricalIndices(cfg));
  auto w = std::make_unique<DatasetWrapper>();
  w->cfg = cfg;
  w->ds = std::make_unique<Dataset>();
  w->ds->InitEmptyLike(ref, num_local_row);
  *out = w.release();
  API_END();
}

int LGBM_DatasetPushRowsByCSRWithMetadata(DatasetHandle dataset, const void* indptr, int indptr_type,
                                          const int32_t* indices, const void* data, int data_type, int64_t nindptr,
                                          int64_t nelem, int64_t start_row, const float* label, const float* weight,
                                          const double* init_score, const int32_t* query, int32_t tid) {
  API_BEGIN();
  (void)tid;
  CSRSource src(indptr, indptr_type == C_API_DTYPE_INT64, indices, data, data_type == C_API_DTYPE_FLOAT64, nindptr,
                nelem, D(dataset)->ds->num_total_features());
  Dataset* ds = D(dataset)->ds.get();
  ds->PushRows(src, static_cast<data_size_t>(start_row));
  const data_size_t n = src.num_rows();
  ds->metadata().SetRows(static_cast<data_size_t>(start_row), n, label, weight, init_score, query);
  API_END();
}

int LGBM_DatasetSerializeReferenceToBinary(DatasetHandle handle, ByteBufferHandle* out, int32_t* out_len) {
  API_BEGIN();
  Dataset empty;
  empty.InitEmptyLike(*D(handle)->ds, 0);
  auto bb = std::make_unique<ByteBuffer>();
  empty.SerializeBinary(&bb->data);
  *out_len = static_cast<int32_t>(bb->data.size());
  *out = bb.release();
  API_END();
}

int LGBM_DatasetCreateFromSerializedReference(const void* ref_buffer, int32_t ref_buffer_size, int64_t num_row,
                                              int32_t num_classes, const char* parameters, DatasetHandle* out) {
  API_BEGIN();
  (void)num_classes;
  auto ref = Dataset::DeserializeBinary(static_cast<const char*>(ref_buffer), static_cast<size_t>(ref_buffer_size));
  auto w = std::make_unique<DatasetWrapper>();
  w->cfg = ParseConfig(parameters);
  w->ds = std::make_unique<Dataset>();
  w->ds->InitEmptyLike(*ref, static_cast<data_size_t>(num_row));
  *out = w.release();
  API_END();
}

int LGBM_ByteBufferGetAt(ByteBufferHandle handle, int32_t index, uint8_t* out_val) {
  API_BEGIN();
  *out_val = static_cast<uint8_t>(static_cast<ByteBuffer*>(handle)->data.at(index));
  API_END();
}

int LGBM_ByteBufferFree(ByteBufferHandle handle) {
  API_BEGIN();
  delete static_cast<ByteBuffer*>(handle);
  API_END();
}

int LGBM_BoosterPredictForMatSingleRowFastInit(BoosterHandle handle, const int predict_type, const int start_iteration,
                                               const int num_iteration, const int data_type, const int32_t ncol,
                                               const char* parameter, FastConfigHandle* out_fastConfig) {
  API_BEGIN();
  *out_fastConfig = MakeFast(handle, predict_type, start_iteration, num_iteration, data_type, ncol, parameter);
  API_END();
}

int LGBM_BoosterPredictForMatSingleRowFast(FastConfigHandle fastConfig_handle, const void* data, int64_t* out_len,
                                           double* out_result) {
  API_BEGIN();
  auto* fc = static_cast<FastConfig*>(fastConfig_handle);
  thread_local std::vector<std::pair<int, double>> row;
  DenseSource src(data, fc->data_type == C_API_DTYPE_FLOAT64, 1, static_cast<int>(fc->ncol), true);
  src.GetRow(0, &row);
  PredictOneRow(fc, row, out_len, out_result);
  API_END();
}

int LGBM_BoosterPredictForCSRSingleRowFastInit(BoosterHandle handle, const int predict_type, const int start_iteration,
                                               const int num_iteration, const int data_type, const int64_t num_col,
                                               const char* parameter, FastConfigHandle* out_fastConfig) {
  API_BEGIN();
  *out_fastConfig = MakeFast(handle, predict_type, start_iteration, num_iteration, data_type, num_col, parameter);
  API_END();
}

int LGBM_BoosterPredictForCSRSingleRowFast(FastConfigHandle fastConfig_handle, const void* indptr,
                                           const int indptr_type, const int32_t* indices, const void* data,
                                           const int64_t nindptr, const int64_t nelem, int64_t* out_len,
                                           double* out_result) {
  API_BEGIN();
  auto* fc = static_cast<FastConfig*>(fastConfig_handle);
  thread_local std::vector<std::pair<int, double>> row;
  CSRSource src(indptr, indptr_type == C_API_DTYPE_INT64, indices, data, fc->data_type == C_API_DTYPE_FLOAT64,
                nindptr, nelem, fc->ncol);
  src.GetRow(0, &row);
  PredictOneRow(fc, row, out_len, out_result);
  API_END();
}

int LGBM_FastConfigFree(FastConfigHandle fastConfig) {
  API_BEGIN();
  delete static_cast<FastConfig*>(fastConfig);
  API_END();
}

int LGBM_BoosterPredictSparseOutput(BoosterHandle handle, const void* indptr, int indptr_type, const int32_t* indices,
                                    const void* data, int data_type, int64_t nindptr, int64_t nelem,
                                    int64_t num_col_or_row, int predict_type, int start_iteration, int num_iteration,
                                    const char* parameter, int matrix_type, int64_t* out_len, void** out_indptr,
                                    int32_t** out_indices, void** out_data) {
  API_BEGIN();
  if (predict_type != C_API_PREDICT_CONTRIB) Log::Fatal("Sparse output is only supported for feature contributions");
  Booster* b = B(handle);
  std::unique_ptr<RowSource> src;
  std::unique_ptr<OwnedSparseSource> csc_rows;
  if (matrix_type == C_API_MATRIX_TYPE_CSR) {
    src = std::make_unique<CSRSource>(indptr, indptr_type == C_API_DTYPE_INT64, indices, data,
                                      data_type == C_API_DTYPE_FLOAT64, nindptr, nelem, num_col_or_row);
  } else if (matrix_type == C_API_MATRIX_TYPE_CSC) {
    csc_rows = CSCToRows(indptr, indptr_type, indices, data, data_type, nindptr, num_col_or_row);
  } else {
    Log::Fatal("Unknown matrix type in LGBM_BoosterPredictSparseOutput");
  }
  const RowSource& rows = csc_rows ? static_cast<const RowSource&>(*csc_rows) : *src;
  const data_size_t nrow = rows.num_rows();
  const int64_t ncol_in = matrix_type == C_API_MATRIX_TYPE_CSR ? num_col_or_row : nindptr - 1;
  GBDT* g = b->boosting_.get();
  const int K = g->NumModelPerIteration();
  const int width = g->MaxFeatureIdx() + 2;  // contributions + expected value
  std::vector<double> dense(static_cast<size_t>(nrow) * K * width);
  int64_t dlen = 0;
  PredictRows(b, rows, predict_type, start_iteration, num_iteration, parameter, &dlen, dense.data());
  // per class matrix: non-zero entries of each row (CSR) or column (CSC)
  const bool i32 = indptr_type == C_API_DTYPE_INT32, f32 = data_type == C_API_DTYPE_FLOAT32;
  const int64_t outer = matrix_type == C_API_MATRIX_TYPE_CSR ? nrow : width;
  const int64_t ptr_len = K * (outer + 1);
  std::vector<int64_t> ptr(ptr_len);
  std::vector<int32_t> idx;
  std::vector<double> val;
  (void)ncol_in;
  for (int k = 0; k < K; ++k) {
    const int64_t base = k * (outer + 1);
    ptr[base] = 0;
    const int64_t start = static_cast<int64_t>(idx.size());
    for (int64_t o = 0; o < outer; ++o) {
      const int64_t inner_n = matrix_type == C_API_MATRIX_TYPE_CSR ? width : nrow;
      for (int64_t q = 0; q < inner_n; ++q) {
        const int64_t r = matrix_type == C_API_MATRIX_TYPE_CSR ? o : q;
        const int64_t c = matrix_type == C_API_MATRIX_TYPE_CSR ? q : o;
        const double v = dense[(static_cast<size_t>(r) * K + k) * width + c];
        if (v != 0.0) {
          idx.push_back(static_cast<int32_t>(q));
          val.push_back(v);
        }
      }
      ptr[base + o + 1] = static_cast<int64_t>(idx.size()) - start;
    }
  }
  if (i32) {
    auto* p = new int32_t[ptr_len];
    for (int64_t i = 0; i < ptr_len; ++i) p[i] = static_cast<int32_t>(ptr[i]);
    *out_indptr = p;
  } else {
    auto* p = new int64_t[ptr_len];
    std::copy(ptr.begin(), ptr.end(), p);
    *out_indptr = p;
  }
  *out_indices = new int32_t[std::max<size_t>(1, idx.size())];
  std::copy(idx.begin(), idx.end(), *out_indices);
  if (f32) {
    auto* d = new float[std::max<size_t>(1, val.size())];
    for (size_t i = 0; i < val.size(); ++i) d[i] = static_cast<float>(val[i]);
    *out_data = d;
  } else {
    auto* d = new double[std::max<size_t>(1, val.size())];
    std::copy(val.begin(), val.end(), d);
    *out_data = d;
  }
  out_len[0] = static_cast<int64_t>(val.size());
  out_len[1] = ptr_len;
  API_END();
}

int LGBM_BoosterFreePredictSparse(void* indptr, int32_t* indices, void* data, int indptr_type, int data_type) {
  API_BEGIN();
  if (indptr_type == C_API_DTYPE_INT32) delete[] static_cast<int32_t*>(indptr);
  else delete[] static_cast<int64_t*>(indptr);
  delete[] indices;
  if (data_type == C_API_DTYPE_FLOAT32) delete[] static_cast<float*>(data);
  else delete[] static_cast<double*>(data);
  API_END();
}
