// Model text format v4 (save / load / JSON dump / C++ if-else codegen),
// feature importance, and raw-feature prediction incl. prediction early
// stopping. Reference: src/boosting/gbdt_model_text.cpp:19-661,
// gbdt_prediction.cpp:13-97, prediction_early_stop.cpp:14-91.
#include <omp.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <sstream>

#include "lgap/boosting.h"
#include "lgap/common.h"
#include "lgap/log.h"

namespace lgap {

// ---------------------------------------------------------------------------
PredictionEarlyStop::PredictionEarlyStop(const std::string& type, int round_period, double margin)
    : round_period_(round_period), margin_(margin) {
  if (type == "none") type_ = 0;
  else if (type == "binary") type_ = 1;
  else if (type == "multiclass") type_ = 2;
  else Log::Fatal("Unknown early stopping type: %s", type.c_str());
}

bool PredictionEarlyStop::Check(const double* pred, int n) const {
  if (type_ == 1) {
    if (n != 1) Log::Fatal("Binary early stopping needs predictions to be of length one");
    return 2.0 * std::fabs(pred[0]) > margin_;
  }
  if (type_ == 2) {
    if (n < 2) Log::Fatal("Multiclass early stopping needs predictions to be of length two or larger");
    std::vector<double> v(pred, pred + n);
    std::partial_sort(v.begin(), v.begin() + 2, v.end(), std::greater<double>());
    return v[0] - v[1] > margin_;
  }
  return false;
}

// ---------------------------------------------------------------------------
void GBDT::InitPredict(int start_iteration, int num_iteration, bool is_pred_contrib) {
  const int total = static_cast<int>(models_.size()) / std::max(1, num_tree_per_iteration_);
  start_iteration = std::max(0, std::min(start_iteration, total));
  num_iteration_for_pred_ = total - start_iteration;
  if (num_iteration > 0) num_iteration_for_pred_ = std::min(num_iteration, num_iteration_for_pred_);
  start_iteration_for_pred_ = start_iteration;
  if (is_pred_contrib) {
    for (auto& m : models_) m->RecomputeMaxDepth();
  }
}

int GBDT::NumPredictOneRow(int start_iteration, int num_iteration, bool is_pred_leaf, bool is_pred_contrib) const {
  int n = num_class_;
  if (objective_ != nullptr) n = objective_->NumPredictOneRow();
  if (is_pred_leaf) {
    const int total = static_cast<int>(models_.size()) / std::max(1, num_tree_per_iteration_);
    start_iteration = std::max(0, std::min(start_iteration, total));
    int iters = total - start_iteration;
    if (num_iteration > 0) iters = std::min(num_iteration, iters);
    return iters * num_tree_per_iteration_;
  }
  if (is_pred_contrib) return num_tree_per_iteration_ * (max_feature_idx_ + 2);
  return n;
}

void GBDT::PredictRaw(const double* x, double* out, const PredictionEarlyStop* es) const {
  std::fill(out, out + num_tree_per_iteration_, 0.0);
  const int end = start_iteration_for_pred_ + num_iteration_for_pred_;
  int counter = 0;
  for (int i = start_iteration_for_pred_; i < end; ++i) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) out[k] += models_[static_cast<size_t>(i) * num_tree_per_iteration_ + k]->Predict(x);
    ++counter;
    if (es && es->enabled() && counter == es->round_period()) {
      if (es->Check(out, num_tree_per_iteration_)) break;
      counter = 0;
    }
  }
  if (average_output_ && num_iteration_for_pred_ > 0) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) out[k] /= num_iteration_for_pred_;
  }
}

void GBDT::PredictRawByMap(const std::unordered_map<int, double>& f, double* out) const {
  std::fill(out, out + num_tree_per_iteration_, 0.0);
  const int end = start_iteration_for_pred_ + num_iteration_for_pred_;
  for (int i = start_iteration_for_pred_; i < end; ++i)
    for (int k = 0; k < num_tree_per_iteration_; ++k) out[k] += models_[static_cast<size_t>(i) * num_tree_per_iteration_ + k]->PredictByMap(f);
  if (average_output_ && num_iteration_for_pred_ > 0)
    for (int k = 0; k < num_tree_per_iteration_; ++k) out[k] /= num_iteration_for_pred_;
}

void GBDT::Predict(const double* x, double* out, const PredictionEarlyStop* es) const {
  std::vector<double> raw(num_tree_per_iteration_);
  PredictRaw(x, raw.data(), es);
  if (objective_ != nullptr) objective_->ConvertOutput(raw.data(), out);
  else std::copy(raw.begin(), raw.end(), out);
}

void GBDT::PredictLeafIndex(const double* x, double* out) const {
  const int end = start_iteration_for_pred_ + num_iteration_for_pred_;
  int p = 0;
  for (int i = start_iteration_for_pred_; i < end; ++i)
    for (int k = 0; k < num_tree_per_iteration_; ++k)
      out[p++] = models_[static_cast<size_t>(i) * num_tree_per_iteration_ + k]->PredictLeafIndex(x);
}

void GBDT::PredictContrib(const double* x, double* out) const {
  const int nf = max_feature_idx_ + 1;
  std::fill(out, out + static_cast<size_t>(num_tree_per_iteration_) * (nf + 1), 0.0);
  const int end = start_iteration_for_pred_ + num_iteration_for_pred_;
  for (int i = start_iteration_for_pred_; i < end; ++i)
    for (int k = 0; k < num_tree_per_iteration_; ++k)
      models_[static_cast<size_t>(i) * num_tree_per_iteration_ + k]->PredictContrib(x, nf, out + static_cast<size_t>(k) * (nf + 1));
}

// ---------------------------------------------------------------------------
std::vector<double> GBDT::FeatureImportance(int num_iteration, int importance_type) const {
  int used = static_cast<int>(models_.size());
  if (num_iteration > 0) used = std::min(num_iteration * num_tree_per_iteration_, used);
  std::vector<double> imp(max_feature_idx_ + 1, 0.0);
  for (int i = 0; i < used; ++i) {
    const Tree* t = models_[i].get();
    for (int n = 0; n < t->num_leaves() - 1; ++n) {
      // only splits that gained count, for both types (reference gbdt_model_text.cpp:635-653)
      if (t->split_gain(n) > 0) {
        if (importance_type == 0) imp[t->split_feature(n)] += 1.0;
        else imp[t->split_feature(n)] += t->split_gain(n);
      }
    }
  }
  return imp;
}

std::string GBDT::SaveModelToString(int start_iteration, int num_iteration, int importance_type) const {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss << SubModelName() << '\n';
  ss << "version=" << kModelVersion << '\n';
  ss << "num_class=" << num_class_ << '\n';
  ss << "num_tree_per_iteration=" << num_tree_per_iteration_ << '\n';
  ss << "label_index=" << label_idx_ << '\n';
  ss << "max_feature_idx=" << max_feature_idx_ << '\n';
  if (objective_ != nullptr) ss << "objective=" << objective_->ToString() << '\n';
  if (average_output_) ss << "average_output" << '\n';
  ss << "feature_names=" << common::Join(feature_names_, " ") << '\n';
  if (!monotone_constraints_.empty()) {
    std::vector<int> mc(monotone_constraints_.begin(), monotone_constraints_.end());
    ss << "monotone_constraints=" << common::Join(mc, " ") << '\n';
  }
  ss << "feature_infos=" << common::Join(feature_infos_, " ") << '\n';
  int used = static_cast<int>(models_.size());
  const int total_iter = used / std::max(1, num_tree_per_iteration_);
  start_iteration = std::max(0, std::min(start_iteration, total_iter));
  if (num_iteration > 0) used = std::min((start_iteration + num_iteration) * num_tree_per_iteration_, used);
  const int start_model = start_iteration * num_tree_per_iteration_;
  std::vector<std::string> strs(std::max(0, used - start_model));
  std::vector<size_t> sizes(strs.size());
#pragma omp parallel for schedule(static)
  for (int i = start_model; i < used; ++i) {
    const int j = i - start_model;
    strs[j] = "Tree=" + std::to_string(j) + "\n" + models_[i]->ToString() + "\n";
    sizes[j] = strs[j].size();
  }
  ss << "tree_sizes=" << common::Join(sizes, " ") << '\n' << '\n';
  for (auto& s : strs) ss << s;
  ss << "end of trees" << '\n';
  auto imp = FeatureImportance(num_iteration, importance_type);
  std::vector<std::pair<size_t, std::string>> pairs;
  for (size_t i = 0; i < imp.size(); ++i) {
    const size_t v = static_cast<size_t>(imp[i]);
    if (v > 0) pairs.emplace_back(v, feature_names_[i]);
  }
  std::stable_sort(pairs.begin(), pairs.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  ss << '\n' << "feature_importances:" << '\n';
  for (auto& p : pairs) ss << p.second << "=" << p.first << '\n';
  if (config_ != nullptr) {
    ss << "\nparameters:" << '\n' << config_->ToString() << "\n" << "end of parameters" << '\n';
  } else if (!loaded_parameter_.empty()) {
    ss << "\nparameters:" << '\n' << loaded_parameter_ << "\n" << "end of parameters" << '\n';
  }
  if (!parser_config_str_.empty()) ss << "\nparser:" << '\n' << parser_config_str_ << "\n" << "end of parser" << '\n';
  return ss.str();
}

bool GBDT::SaveModelToFile(int start_iteration, int num_iteration, int importance_type, const std::string& fn) const {
  std::ofstream out(fn, std::ios::binary);
  if (!out) Log::Fatal("Model file %s is not available for writes", fn.c_str());
  std::string s = SaveModelToString(start_iteration, num_iteration, importance_type);
  out.write(s.data(), s.size());
  return static_cast<bool>(out);
}

bool GBDT::LoadModelFromString(const char* buffer, size_t len) {
  models_.clear();
  const char* p = buffer;
  const char* end = buffer + len;
  std::unordered_map<std::string, std::string> kv;
  // header: until the first "Tree=" line
  while (p < end) {
    const char* e = p;
    while (e < end && *e != '\n' && *e != '\r') ++e;
    std::string line(p, e - p);
    if (common::StartsWith(line, "Tree=") || line == "end of trees") break;
    if (!line.empty()) {
      size_t eq = line.find('=');
      if (eq == std::string::npos) kv[line] = "";
      else kv[line.substr(0, eq)] = line.substr(eq + 1);
    }
    p = e;
    while (p < end && (*p == '\n' || *p == '\r')) ++p;
  }
  if (!kv.count("num_class")) Log::Fatal("Model file doesn't specify the number of classes");
  num_class_ = common::AtoiOrDie(kv["num_class"]);
  num_tree_per_iteration_ = kv.count("num_tree_per_iteration") ? common::AtoiOrDie(kv["num_tree_per_iteration"]) : num_class_;
  label_idx_ = kv.count("label_index") ? common::AtoiOrDie(kv["label_index"]) : 0;
  if (!kv.count("max_feature_idx")) Log::Fatal("Model file doesn't specify max_feature_idx");
  max_feature_idx_ = common::AtoiOrDie(kv["max_feature_idx"]);
  average_output_ = kv.count("average_output") > 0;
  feature_names_ = kv.count("feature_names") ? common::Split(kv["feature_names"], ' ') : std::vector<std::string>();
  if (static_cast<int>(feature_names_.size()) != max_feature_idx_ + 1) {
    Log::Fatal("Wrong size of feature_names");
  }
  monotone_constraints_.clear();
  if (kv.count("monotone_constraints")) {
    for (auto& s : common::Split(kv["monotone_constraints"], ' ')) monotone_constraints_.push_back(static_cast<int8_t>(common::AtoiOrDie(s)));
  }
  feature_infos_ = kv.count("feature_infos") ? common::Split(kv["feature_infos"], ' ') : std::vector<std::string>();
  if (kv.count("objective")) {
    loaded_objective_ = ObjectiveFunction::CreateFromString(kv["objective"]);
    objective_ = loaded_objective_.get();
  } else {
    objective_ = nullptr;
  }
  // trees
  while (p < end) {
    const char* e = p;
    while (e < end && *e != '\n' && *e != '\r') ++e;
    std::string line(p, e - p);
    if (line == "end of trees") {
      p = e;
      break;
    }
    if (common::StartsWith(line, "Tree=")) {
      p = e;
      while (p < end && (*p == '\n' || *p == '\r')) ++p;
      // tree block ends at the next blank-line-separated "Tree=" / "end of trees"
      const char* q = p;
      while (q < end) {
        const char* qe = q;
        while (qe < end && *qe != '\n' && *qe != '\r') ++qe;
        std::string l(q, qe - q);
        if (common::StartsWith(l, "Tree=") || l == "end of trees") break;
        q = qe;
        while (q < end && (*q == '\n' || *q == '\r')) ++q;
      }
      std::string block(p, q - p);
      size_t used;
      models_.push_back(std::make_unique<Tree>(block.c_str(), &used));
      p = q;
      continue;
    }
    p = e;
    while (p < end && (*p == '\n' || *p == '\r')) ++p;
  }
  Log::Info("Finished loading %d models", static_cast<int>(models_.size()));
  num_iteration_for_pred_ = static_cast<int>(models_.size()) / std::max(1, num_tree_per_iteration_);
  start_iteration_for_pred_ = 0;
  // parameters
  const char* ps = std::strstr(p, "\nparameters:");
  if (ps == nullptr && std::strncmp(p, "parameters:", 11) == 0) ps = p - 1;
  if (ps != nullptr && ps < end) {
    const char* b = ps + std::strlen("\nparameters:");
    while (b < end && (*b == '\n' || *b == '\r')) ++b;
    const char* pe = std::strstr(b, "end of parameters");
    if (pe != nullptr) {
      loaded_parameter_ = std::string(b, pe - b);
      while (!loaded_parameter_.empty() && (loaded_parameter_.back() == '\n' || loaded_parameter_.back() == '\r'))
        loaded_parameter_.pop_back();
    }
  }
  const char* pp = std::strstr(p, "\nparser:");
  if (pp != nullptr && pp < end) {
    const char* b = pp + std::strlen("\nparser:\n");
    const char* pe = std::strstr(b, "end of parser");
    if (pe != nullptr) parser_config_str_ = common::Trim(std::string(b, pe - b));
  }
  return true;
}

std::string GBDT::DumpModel(int start_iteration, int num_iteration, int importance_type) const {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss << "{";
  ss << "\"name\":\"" << SubModelName() << "\",\n";
  ss << "\"version\":\"" << kModelVersion << "\",\n";
  ss << "\"num_class\":" << num_class_ << ",\n";
  ss << "\"num_tree_per_iteration\":" << num_tree_per_iteration_ << ",\n";
  ss << "\"label_index\":" << label_idx_ << ",\n";
  ss << "\"max_feature_idx\":" << max_feature_idx_ << ",\n";
  if (objective_ != nullptr) ss << "\"objective\":\"" << objective_->ToString() << "\",\n";
  ss << "\"average_output\":" << (average_output_ ? "true" : "false") << ",\n";
  ss << "\"feature_names\":[\"" << common::Join(feature_names_, "\",\"") << "\"],\n";
  std::vector<int> mc(monotone_constraints_.begin(), monotone_constraints_.end());
  ss << "\"monotone_constraints\":[" << common::Join(mc, ",") << "],\n";
  ss << "\"feature_infos\":{";
  bool first = true;
  for (size_t i = 0; i < feature_infos_.size(); ++i) {
    const std::string& fi = feature_infos_[i];
    std::stringstream js;
    js.imbue(std::locale::classic());
    js << std::setprecision(std::numeric_limits<double>::digits10 + 2);
    if (!fi.empty() && fi[0] == '[') {
      auto parts = common::Split(fi.substr(1, fi.size() - 2), ':');
      double mn = common::AtofOrDie(parts[0]), mx = common::AtofOrDie(parts[1]);
      js << "{\"min_value\":" << common::AvoidInf(mn) << ",\"max_value\":" << common::AvoidInf(mx) << ",\"values\":[]}";
    } else if (fi != "none") {
      std::vector<int> vals;
      for (auto& s : common::Split(fi, ':')) vals.push_back(common::AtoiOrDie(s));
      js << "{\"min_value\":" << *std::min_element(vals.begin(), vals.end()) << ",\"max_value\":"
         << *std::max_element(vals.begin(), vals.end()) << ",\"values\":[" << common::Join(vals, ",") << "]}";
    } else {
      continue;
    }
    if (!first) ss << ",";
    ss << "\"" << feature_names_[i] << "\":" << js.str();
    first = false;
  }
  ss << "},\n";
  ss << "\"tree_info\":[";
  int used = static_cast<int>(models_.size());
  const int total_iter = used / std::max(1, num_tree_per_iteration_);
  start_iteration = std::max(0, std::min(start_iteration, total_iter));
  if (num_iteration > 0) used = std::min((start_iteration + num_iteration) * num_tree_per_iteration_, used);
  const int start_model = start_iteration * num_tree_per_iteration_;
  for (int i = start_model; i < used; ++i) {
    if (i > start_model) ss << ",";
    ss << "{\"tree_index\":" << i << "," << models_[i]->ToJSON() << "}";
  }
  ss << "],\n";
  auto imp = FeatureImportance(num_iteration, importance_type);
  std::vector<std::pair<size_t, std::string>> pairs;
  for (size_t i = 0; i < imp.size(); ++i) {
    const size_t v = static_cast<size_t>(imp[i]);
    if (v > 0) pairs.emplace_back(v, feature_names_[i]);
  }
  std::stable_sort(pairs.begin(), pairs.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  ss << "\n\"feature_importances\":{";
  for (size_t i = 0; i < pairs.size(); ++i) ss << (i ? "," : "") << "\"" << pairs[i].second << "\":" << pairs[i].first;
  ss << "}\n}\n";
  return ss.str();
}

std::string GBDT::ModelToIfElse(int num_iteration) const {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss << "#include <cmath>\n#include <cstdint>\n#include <cstring>\n\n";
  ss << "namespace lambdagap_generated {\n\n";
  int used = static_cast<int>(models_.size());
  if (num_iteration > 0) used = std::min(num_iteration * num_tree_per_iteration_, used);
  for (int i = 0; i < used; ++i) ss << models_[i]->ToIfElse(i, false);
  for (int i = 0; i < used; ++i) ss << models_[i]->ToIfElse(i, true);
  ss << "\ntypedef double (*PredictFn)(const double*);\n";
  ss << "static const PredictFn kPredictTree[] = {";
  for (int i = 0; i < used; ++i) ss << (i ? ", " : "") << "PredictTree" << i;
  ss << "};\n";
  ss << "static const PredictFn kPredictTreeLeaf[] = {";
  for (int i = 0; i < used; ++i) ss << (i ? ", " : "") << "PredictTree" << i << "Leaf";
  ss << "};\n\n";
  ss << "const int kNumTreePerIteration = " << num_tree_per_iteration_ << ";\n";
  ss << "const int kNumModels = " << used << ";\n";
  ss << "void PredictRaw(const double* features, double* output) {\n";
  ss << "  for (int k = 0; k < kNumTreePerIteration; ++k) output[k] = 0.0;\n";
  ss << "  for (int i = 0; i < kNumModels; ++i) output[i % kNumTreePerIteration] += kPredictTree[i](features);\n";
  if (average_output_) ss << "  for (int k = 0; k < kNumTreePerIteration; ++k) output[k] /= (kNumModels / kNumTreePerIteration);\n";
  ss << "}\n";
  ss << "void PredictLeafIndex(const double* features, double* output) {\n";
  ss << "  for (int i = 0; i < kNumModels; ++i) output[i] = kPredictTreeLeaf[i](features);\n}\n";
  ss << "}  // namespace lambdagap_generated\n";
  return ss.str();
}

}  // namespace lgap
