// CLI application: `lambdagap config=train.conf [key=value ...]`
// Tasks: train, predict, convert_model, refit, save_binary
// (reference: src/main.cpp, src/application/application.cpp:31-291).
#include <omp.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <vector>

#include "lgap/omp_errors.h"
#include "lgap/threading.h"
#include "lgap/boosting.h"
#include "lgap/common.h"
#include "lgap/config.h"
#include "lgap/dataset.h"
#include "lgap/log.h"
#include "lgap/metric.h"
#include "lgap/network.h"
#include "lgap/objective.h"

using namespace lgap;

namespace {

ParamMap LoadParameters(int argc, char** argv) {
  std::unordered_map<std::string, std::vector<std::string>> all;
  for (int i = 1; i < argc; ++i) Config::KV2Map(&all, argv[i]);
  ParamMap params;
  for (auto& kv : all) params[kv.first] = kv.second[0];
  Config::KeyAliasTransform(&params);
  if (params.count("config")) {
    std::ifstream in(params["config"]);
    if (!in) Log::Fatal("Config file %s doesn't exist", params["config"].c_str());
    std::unordered_map<std::string, std::vector<std::string>> fa;
    std::string line;
    while (std::getline(in, line)) {
      line = common::Trim(line);
      if (line.empty() || line[0] == '#') continue;
      Config::KV2Map(&fa, line.c_str());
    }
    ParamMap fp;
    for (auto& kv : fa) fp[kv.first] = kv.second[0];
    Config::KeyAliasTransform(&fp);
    for (auto& kv : fp) {
      if (!params.count(kv.first)) params[kv.first] = kv.second;  // command line wins
    }
  }
  return params;
}

std::vector<std::unique_ptr<Metric>> MakeMetrics(const Config& c, const Dataset& d) {
  std::vector<std::unique_ptr<Metric>> out;
  for (auto& m : c.metric) {
    auto met = Metric::Create(m, c);
    if (!met) continue;
    met->Init(d.metadata(), d.num_data());
    out.push_back(std::move(met));
  }
  return out;
}

std::vector<const Metric*> Ptrs(const std::vector<std::unique_ptr<Metric>>& v) {
  std::vector<const Metric*> o;
  for (auto& m : v) o.push_back(m.get());
  return o;
}

void Predict(const Config& c) {
  auto boosting = CreateBoosting("gbdt", c.input_model.c_str());
  OwnedSparseSource rows;
  std::vector<float> labels;
  int label_idx = 0;
  if (!c.label_column.empty() && !common::StartsWith(c.label_column, "name:")) label_idx = common::AtoiOrDie(c.label_column);
  ParseTextFile(c.data, c.header, label_idx, &rows, &labels, nullptr, nullptr, {}, -1, nullptr, -1, nullptr);
  const bool leaf = c.predict_leaf_index, contrib = c.predict_contrib, raw = c.predict_raw_score;
  boosting->InitPredict(c.start_iteration_predict, c.num_iteration_predict, contrib);
  const int per = boosting->NumPredictOneRow(c.start_iteration_predict, c.num_iteration_predict, leaf, contrib);
  const int nf = std::max(boosting->MaxFeatureIdx() + 1, rows.ncol);
  std::vector<double> out(rows.rows.size() * static_cast<size_t>(per));
  std::string es_type = "none";
  if (c.pred_early_stop && !leaf && !contrib && !boosting->NeedAccuratePrediction()) {
    es_type = boosting->NumberOfClasses() == 1 ? "binary" : "multiclass";
  }
  PredictionEarlyStop es(es_type, c.pred_early_stop_freq, c.pred_early_stop_margin);
  OmpErrors errs;
#pragma omp parallel
  {
    std::vector<double> x(nf);
#pragma omp for schedule(static)
    for (size_t i = 0; i < rows.rows.size(); ++i) {
      errs.Run([&] {
        std::fill(x.begin(), x.end(), 0.0);
        for (auto& kv : rows.rows[i]) if (kv.first < nf) x[kv.first] = kv.second;
        double* o = out.data() + i * per;
        if (leaf) boosting->PredictLeafIndex(x.data(), o);
        else if (contrib) boosting->PredictContrib(x.data(), o);
        else if (raw) boosting->PredictRaw(x.data(), o, nullptr);
        else boosting->Predict(x.data(), o, &es);
      });
    }
  }
  errs.Rethrow();
  std::ofstream fo(c.output_result);
  for (size_t i = 0; i < rows.rows.size(); ++i) {
    for (int k = 0; k < per; ++k) fo << (k ? "\t" : "") << common::Format17(out[i * per + k]);
    fo << '\n';
  }
  Log::Info("Finished prediction");
}

void Train(Config& c) {
  if (c.num_machines > 1) {
    Network::Init(c);
    c.seed = Network::GlobalSyncUpByMin(c.seed);
    c.data_random_seed = Network::GlobalSyncUpByMin(c.data_random_seed);
    c.bagging_seed = Network::GlobalSyncUpByMin(c.bagging_seed);
    c.feature_fraction_seed = Network::GlobalSyncUpByMin(c.feature_fraction_seed);
  }
  auto train = LoadDatasetFromFile(c.data, c, nullptr, Network::rank(), Network::num_machines());
  std::vector<std::unique_ptr<Dataset>> valids;
  for (auto& v : c.valid) valids.push_back(LoadDatasetFromFile(v, c, train.get(), 0, 1));
  auto boosting = CreateBoosting(c.boosting, c.input_model.c_str());
  auto objective = ObjectiveFunction::Create(c.objective, c);
  if (objective) objective->Init(train->metadata(), train->num_data());
  std::vector<std::unique_ptr<Metric>> train_metrics;
  if (c.is_provide_training_metric) train_metrics = MakeMetrics(c, *train);
  boosting->Init(&c, train.get(), objective.get(), Ptrs(train_metrics));
  std::vector<std::vector<std::unique_ptr<Metric>>> vm;
  for (auto& v : valids) {
    vm.push_back(MakeMetrics(c, *v));
    boosting->AddValidDataset(v.get(), Ptrs(vm.back()));
  }
  auto t0 = std::chrono::steady_clock::now();
  boosting->Train(c.snapshot_freq, c.output_model);
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (Network::rank() == 0 || c.num_machines <= 1) {
    boosting->SaveModelToFile(0, -1, c.saved_feature_importance_type, c.output_model);
    if (c.convert_model_language == "cpp") {
      std::ofstream f(c.convert_model);
      f << boosting->ModelToIfElse(-1);
    }
  }
  Log::Info("Finished training in %f seconds", sec);
}

void ConvertModel(const Config& c) {
  auto boosting = CreateBoosting("gbdt", c.input_model.c_str());
  std::ofstream f(c.convert_model);
  f << boosting->ModelToIfElse(c.num_iteration_predict);
  Log::Info("Converted model to %s", c.convert_model.c_str());
}

void SaveBinary(Config& c) {
  auto train = LoadDatasetFromFile(c.data, c, nullptr, 0, 1);
  train->SaveBinary(c.data + ".bin");
  for (auto& v : c.valid) {
    auto vd = LoadDatasetFromFile(v, c, train.get(), 0, 1);
    vd->SaveBinary(v + ".bin");
  }
}

void Refit(Config& c) {
  auto boosting = CreateBoosting("gbdt", c.input_model.c_str());
  auto train = LoadDatasetFromFile(c.data, c, nullptr, 0, 1);
  // leaf predictions of the existing model on the raw training file
  OwnedSparseSource rows;
  std::vector<float> labels;
  ParseTextFile(c.data, c.header, 0, &rows, &labels, nullptr, nullptr, {}, -1, nullptr, -1, nullptr);
  boosting->InitPredict(0, -1, false);
  const int per = boosting->NumPredictOneRow(0, -1, true, false);
  const int nf = std::max(boosting->MaxFeatureIdx() + 1, rows.ncol);
  std::vector<std::vector<int>> lp(rows.rows.size(), std::vector<int>(per));
  std::vector<double> x(nf), o(per);
  for (size_t i = 0; i < rows.rows.size(); ++i) {
    std::fill(x.begin(), x.end(), 0.0);
    for (auto& kv : rows.rows[i]) if (kv.first < nf) x[kv.first] = kv.second;
    boosting->PredictLeafIndex(x.data(), o.data());
    for (int k = 0; k < per; ++k) lp[i][k] = static_cast<int>(o[k]);
  }
  auto fresh = CreateBoosting(c.boosting, nullptr);
  auto objective = ObjectiveFunction::Create(c.objective, c);
  if (objective) objective->Init(train->metadata(), train->num_data());
  fresh->Init(&c, train.get(), objective.get(), {});
  for (int i = 0; i < boosting->NumberOfTotalModel(); ++i) fresh->AddTree(std::make_unique<Tree>(*boosting->GetTree(i)));
  fresh->RefitTree(lp);
  fresh->SaveModelToFile(0, -1, c.saved_feature_importance_type, c.output_model);
}

}  // namespace

int main(int argc, char** argv) {
  try {
    ParamMap params = LoadParameters(argc, argv);
    Config c;
    c.Set(params);
    SetDefaultNumThreads(c.num_threads);
    if (c.task == "train") Train(c);
    else if (c.task == "predict") Predict(c);
    else if (c.task == "convert_model") ConvertModel(c);
    else if (c.task == "save_binary") SaveBinary(c);
    else if (c.task == "refit") Refit(c);
    else Log::Fatal("Unknown task %s", c.task.c_str());
    Network::Dispose();
  } catch (std::exception& e) {
    std::cerr << "Met Exceptions:\n" << e.what() << std::endl;
    Network::Dispose();
    return -1;
  }
  return 0;
}
