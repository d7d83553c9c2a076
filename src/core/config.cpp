// Config parsing: alias resolution, typed getters with range checks, derived
// flags and conflict resolution. Behaviour mirrors src/io/config.cpp of the
// reference; the tables are generated from config_params.def instead of a
// separate code generator.
#include <limits>
#include <map>
#include "lgap/config.h"

#include <algorithm>
#include <cmath>
#include <set>
#include <sstream>
#include <unordered_set>

#include "lgap/common.h"
#include "lgap/log.h"
#include "lgap/random.h"

namespace lgap {

namespace {

struct ParamInfo {
  const char* name;
  const char* kind;
  const char* aliases;
  bool save;
  const char* check;
};

const std::vector<ParamInfo>& ParamTable() {
  static const std::vector<ParamInfo> t = {
#define LGAP_PARAM(kind, name, def, aliases, save, check) {#name, #kind, aliases, save != 0, check},
#include "lgap/config_params.def"
#undef LGAP_PARAM
  };
  return t;
}

void CheckRange(const std::string& name, double v, const std::string& checks) {
  for (auto& c : common::Split(checks, ',')) {
    std::string op;
    size_t i = 0;
    while (i < c.size() && (c[i] == '<' || c[i] == '>' || c[i] == '=')) op.push_back(c[i++]);
    double bound = common::AtofOrDie(c.substr(i));
    bool ok = true;
    if (op == ">") ok = v > bound;
    else if (op == ">=") ok = v >= bound;
    else if (op == "<") ok = v < bound;
    else if (op == "<=") ok = v <= bound;
    if (!ok) Log::Fatal("Parameter %s should be %s, got %g", name.c_str(), c.c_str(), v);
  }
}

bool ParseBool(const std::string& name, std::string v) {
  v = common::ToLower(common::Trim(v));
  if (v == "true" || v == "1" || v == "+" || v == "yes") return true;
  if (v == "false" || v == "0" || v == "-" || v == "no" || v.empty()) return false;
  Log::Fatal("Parameter %s should be of type bool, got \"%s\"", name.c_str(), v.c_str());
}

template <typename T>
std::vector<T> ParseNumVec(const std::string& v) {
  std::vector<T> out;
  for (auto& tok : common::SplitAny(v, ", ")) out.push_back(static_cast<T>(common::AtofOrDie(tok)));
  return out;
}

std::vector<std::vector<int>> ParseArrayOfArrays(const std::string& s) {
  std::vector<std::vector<int>> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t b = s.find('[', i);
    if (b == std::string::npos) break;
    size_t e = s.find(']', b);
    if (e == std::string::npos) Log::Fatal("Malformed interaction_constraints: %s", s.c_str());
    out.push_back(ParseNumVec<int>(s.substr(b + 1, e - b - 1)));
    i = e + 1;
  }
  return out;
}

}  // namespace

const std::unordered_map<std::string, std::string>& Config::AliasTable() {
  static const std::unordered_map<std::string, std::string> table = [] {
    std::unordered_map<std::string, std::string> m;
    for (auto& p : ParamTable()) {
      for (auto& a : common::Split(p.aliases, ',')) m[a] = p.name;
    }
    return m;
  }();
  return table;
}

bool Config::IsKnownParameter(const std::string& name) {
  for (auto& p : ParamTable()) if (name == p.name) return true;
  return AliasTable().count(name) > 0;
}

void Config::KV2Map(std::unordered_map<std::string, std::vector<std::string>>* params, const char* kv) {
  std::string s = common::Trim(kv);
  if (s.empty() || s[0] == '#') return;
  size_t hash = s.find('#');
  if (hash != std::string::npos) s = common::Trim(s.substr(0, hash));
  size_t eq = s.find('=');
  if (eq == std::string::npos) {
    Log::Warning("Unknown parameter %s", s.c_str());
    return;
  }
  std::string key = common::ToLower(common::Trim(s.substr(0, eq)));
  std::string value = common::RemoveQuotes(common::Trim(s.substr(eq + 1)));
  if (key.empty()) return;
  (*params)[key].push_back(value);
}

// Reference config.h ParameterAlias::KeyAliasTransform: among several aliases of one
// parameter the shortest (then alphabetically first) name wins; a canonical name wins over
// any alias. Every loser is reported.
void Config::KeyAliasTransform(ParamMap* params) {
  const auto& alias = AliasTable();
  auto sort_alias = [](const std::string& x, const std::string& y) {
    return x.size() < y.size() || (x.size() == y.size() && x < y);
  };
  std::vector<std::string> keys;
  for (auto& kv : *params) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());
  std::map<std::string, std::string> chosen;  // canonical -> winning alias key
  for (const auto& k : keys) {
    auto it = alias.find(k);
    if (it == alias.end()) {
      if (!IsKnownParameter(k)) Log::Warning("Unknown parameter: %s", k.c_str());
      continue;
    }
    auto c = chosen.find(it->second);
    if (c == chosen.end()) {
      chosen.emplace(it->second, k);
    } else if (sort_alias(c->second, k)) {
      Log::Warning("%s is set with %s=%s, %s=%s will be ignored. Current value: %s=%s", it->second.c_str(),
                   c->second.c_str(), params->at(c->second).c_str(), k.c_str(), params->at(k).c_str(),
                   it->second.c_str(), params->at(c->second).c_str());
    } else {
      Log::Warning("%s is set with %s=%s, will be overridden by %s=%s. Current value: %s=%s", it->second.c_str(),
                   c->second.c_str(), params->at(c->second).c_str(), k.c_str(), params->at(k).c_str(),
                   it->second.c_str(), params->at(k).c_str());
      c->second = k;
    }
  }
  ParamMap out;
  for (auto& kv : *params) {
    if (alias.count(kv.first) == 0) out[kv.first] = kv.second;
  }
  for (auto& kv : chosen) {
    auto canon = out.find(kv.first);
    if (canon == out.end()) {
      out[kv.first] = params->at(kv.second);
    } else {
      Log::Warning("%s is set=%s, %s=%s will be ignored. Current value: %s=%s", kv.first.c_str(),
                   canon->second.c_str(), kv.second.c_str(), params->at(kv.second).c_str(), kv.first.c_str(),
                   canon->second.c_str());
    }
  }
  *params = std::move(out);
}

ParamMap Config::Str2Map(const char* parameters) {
  std::unordered_map<std::string, std::vector<std::string>> all;
  for (auto& arg : common::SplitAny(parameters ? parameters : "", " \t\n\r")) KV2Map(&all, arg.c_str());
  // the log level follows verbose / verbosity before any alias is reported (reference
  // config.cpp SetVerbosity: verbosity over verbose)
  int verbosity = Config().verbosity;
  for (const char* key : {"verbose", "verbosity"}) {
    auto it = all.find(key);
    if (it != all.end()) verbosity = std::atoi(it->second[0].c_str());
  }
  if (verbosity < 0) Log::ResetLevel(LogLevel::Fatal);
  else if (verbosity == 0) Log::ResetLevel(LogLevel::Warning);
  else if (verbosity == 1) Log::ResetLevel(LogLevel::Info);
  else Log::ResetLevel(LogLevel::Debug);
  ParamMap params;
  for (auto& kv : all) {
    params[kv.first] = kv.second[0];
    for (size_t i = 1; i < kv.second.size(); ++i) {
      Log::Warning("%s is set=%s, %s=%s will be ignored. Current value: %s=%s", kv.first.c_str(),
                   kv.second[0].c_str(), kv.first.c_str(), kv.second[i].c_str(), kv.first.c_str(),
                   kv.second[0].c_str());
    }
  }
  KeyAliasTransform(&params);
  return params;
}

std::string ParseObjectiveAlias(const std::string& t) {
  static const std::unordered_map<std::string, std::string> m = {
      {"regression_l2", "regression"}, {"mean_squared_error", "regression"}, {"mse", "regression"},
      {"l2", "regression"}, {"l2_root", "regression"}, {"root_mean_squared_error", "regression"},
      {"rmse", "regression"}, {"mean_absolute_error", "regression_l1"}, {"l1", "regression_l1"},
      {"mae", "regression_l1"}, {"softmax", "multiclass"}, {"multiclass_ova", "multiclassova"},
      {"ova", "multiclassova"}, {"ovr", "multiclassova"}, {"xentropy", "cross_entropy"},
      {"xentlambda", "cross_entropy_lambda"}, {"mean_absolute_percentage_error", "mape"},
      {"xendcg", "rank_xendcg"}, {"xe_ndcg", "rank_xendcg"}, {"xe_ndcg_mart", "rank_xendcg"},
      {"xendcg_mart", "rank_xendcg"}, {"none", "custom"}, {"null", "custom"}, {"na", "custom"}};
  auto it = m.find(t);
  return it == m.end() ? t : it->second;
}

std::string ParseMetricAlias(const std::string& t) {
  static const std::unordered_map<std::string, std::string> m = {
      {"regression", "l2"}, {"regression_l2", "l2"}, {"mean_squared_error", "l2"}, {"mse", "l2"},
      {"l2_root", "rmse"}, {"root_mean_squared_error", "rmse"}, {"regression_l1", "l1"},
      {"mean_absolute_error", "l1"}, {"mae", "l1"}, {"binary", "binary_logloss"}, {"lambdarank", "ndcg"},
      {"rank_xendcg", "ndcg"}, {"xendcg", "ndcg"}, {"xe_ndcg", "ndcg"}, {"xe_ndcg_mart", "ndcg"},
      {"xendcg_mart", "ndcg"}, {"mean_average_precision", "map"}, {"multiclass", "multi_logloss"},
      {"softmax", "multi_logloss"}, {"multiclassova", "multi_logloss"}, {"multiclass_ova", "multi_logloss"},
      {"ova", "multi_logloss"}, {"ovr", "multi_logloss"}, {"xentropy", "cross_entropy"},
      {"xentlambda", "cross_entropy_lambda"}, {"kldiv", "kullback_leibler"},
      {"mean_absolute_percentage_error", "mape"}, {"none", "custom"}, {"null", "custom"}, {"na", "custom"},
      {"precision@k", "precision"}};
  auto it = m.find(t);
  return it == m.end() ? t : it->second;
}

namespace {
// typed parameter values must be the whole string (reference config.h GetInt / GetDouble)
double ParseDblParam(const char* name, const std::string& v) {
  const std::string t = common::Trim(v);
  char* end = nullptr;
  const double d = std::strtod(t.c_str(), &end);
  if (t.empty() || *end != '\0') {
    const std::string l = common::ToLower(t);
    if (l == "inf" || l == "+inf" || l == "infinity") return std::numeric_limits<double>::infinity();
    if (l == "-inf" || l == "-infinity") return -std::numeric_limits<double>::infinity();
    Log::Fatal("Parameter %s should be of type double, got \"%s\"", name, v.c_str());
  }
  return d;
}
int ParseIntParam(const char* name, const std::string& v) {
  const std::string t = common::Trim(v);
  char* end = nullptr;
  const long long i = std::strtoll(t.c_str(), &end, 10);
  if (!t.empty() && *end == '\0') return static_cast<int>(i);
  const double d = std::strtod(t.c_str(), &end);  // integral spellings such as 1e3 or 31.0
  if (t.empty() || *end != '\0' || d != std::floor(d)) {
    Log::Fatal("Parameter %s should be of type int, got \"%s\"", name, v.c_str());
  }
  return static_cast<int>(d);
}
}  // namespace

void Config::GetMembersFromString(const ParamMap& params) {
  auto get = [&](const char* n, std::string* v) {
    auto it = params.find(n);
    if (it == params.end()) return false;
    *v = it->second;
    return true;
  };
  std::string v;
#define LGAP_PARSE_STR(name, check) if (get(#name, &v)) name = v;
#define LGAP_PARSE_INT(name, check) \
  if (get(#name, &v) && !v.empty()) { name = ParseIntParam(#name, v); CheckRange(#name, name, check); }
#define LGAP_PARSE_DBL(name, check) \
  if (get(#name, &v) && !v.empty()) { name = ParseDblParam(#name, v); CheckRange(#name, name, check); }
#define LGAP_PARSE_BOOL(name, check) if (get(#name, &v)) name = ParseBool(#name, v);
#define LGAP_PARSE_VSTR(name, check) if (get(#name, &v)) name = common::Split(v, ',');
#define LGAP_PARSE_VINT(name, check) if (get(#name, &v)) name = ParseNumVec<int>(v);
#define LGAP_PARSE_VDBL(name, check) if (get(#name, &v)) name = ParseNumVec<double>(v);
#define LGAP_PARSE_VI8(name, check) if (get(#name, &v)) name = ParseNumVec<int8_t>(v);
#define LGAP_PARSE_VI32(name, check) if (get(#name, &v)) name = ParseNumVec<int32_t>(v);
#define LGAP_PARAM(kind, name, def, aliases, save, check) LGAP_PARSE_##kind(name, check)
  // objective / metric / boosting etc. are handled specially by Set(); skip them here
  const std::string objective_keep = objective, boosting_keep = boosting;
  const std::vector<std::string> metric_keep = metric;
  const std::string task_keep = task, device_keep = device_type, learner_keep = tree_learner;
  const std::string dss_keep = data_sample_strategy;
#include "lgap/config_params.def"
#undef LGAP_PARAM
  objective = objective_keep;
  boosting = boosting_keep;
  metric = metric_keep;
  task = task_keep;
  device_type = device_keep;
  tree_learner = learner_keep;
  data_sample_strategy = dss_keep;
}

static void ParseMetrics(const std::string& value, std::vector<std::string>* out) {
  std::unordered_set<std::string> seen;
  out->clear();
  for (auto& m : common::Split(value, ',')) {
    auto t = ParseMetricAlias(common::Trim(m));
    if (seen.insert(t).second) out->push_back(t);
  }
}

void Config::Set(const ParamMap& params) {
  auto has = [&](const char* n, std::string* v) {
    auto it = params.find(n);
    if (it == params.end()) return false;
    *v = common::ToLower(common::Trim(it->second));
    return true;
  };
  std::string v;
  if (has("seed", &v) && !v.empty()) {
    seed = static_cast<int>(common::AtofOrDie(v));
    Random rand(seed);
    const int int_max = 32767;
    data_random_seed = rand.NextShort(0, int_max);
    bagging_seed = rand.NextShort(0, int_max);
    drop_seed = rand.NextShort(0, int_max);
    feature_fraction_seed = rand.NextShort(0, int_max);
    objective_seed = rand.NextShort(0, int_max);
    extra_seed = rand.NextShort(0, int_max);
  }
  if (has("task", &v)) {
    if (v == "train" || v == "training") task = "train";
    else if (v == "predict" || v == "prediction" || v == "test") task = "predict";
    else if (v == "convert_model") task = "convert_model";
    else if (v == "refit" || v == "refit_tree") task = "refit";
    else if (v == "save_binary") task = "save_binary";
    else Log::Fatal("Unknown task type %s", v.c_str());
  }
  if (has("boosting", &v)) {
    if (v == "gbdt" || v == "gbrt") boosting = "gbdt";
    else if (v == "dart") boosting = "dart";
    else if (v == "goss") boosting = "goss";
    else if (v == "rf" || v == "random_forest") boosting = "rf";
    else Log::Fatal("Unknown boosting type %s", v.c_str());
  }
  if (has("data_sample_strategy", &v)) {
    if (v == "goss" || v == "bagging") data_sample_strategy = v;
    else Log::Fatal("Unknown sample strategy %s", v.c_str());
  }
  if (has("objective", &v)) objective = ParseObjectiveAlias(v);
  {
    bool got = has("metric", &v);
    if (got) ParseMetrics(v, &metric);
    if (metric.empty() && (!got || v.empty())) ParseMetrics(objective, &metric);
  }
  if (has("device_type", &v)) {
    if (v == "cpu" || v == "gpu" || v == "cuda" || v == "hip" || v == "rocm") {
      device_type = (v == "hip" || v == "rocm") ? "gpu" : v;
    } else {
      Log::Fatal("Unknown device type %s", v.c_str());
    }
  }
  if (has("tree_learner", &v)) {
    if (v == "serial") tree_learner = "serial";
    else if (v == "feature" || v == "feature_parallel") tree_learner = "feature";
    else if (v == "data" || v == "data_parallel") tree_learner = "data";
    else if (v == "voting" || v == "voting_parallel") tree_learner = "voting";
    else Log::Fatal("Unknown tree learner type %s", v.c_str());
  }
  GetMembersFromString(params);

  if (verbosity < 0) Log::ResetLevel(LogLevel::Fatal);
  else if (verbosity == 0) Log::ResetLevel(LogLevel::Warning);
  else if (verbosity == 1) Log::ResetLevel(LogLevel::Info);
  else Log::ResetLevel(LogLevel::Debug);

  // auc_mu weights
  if (auc_mu_weights.empty()) {
    auc_mu_weights_matrix.assign(num_class, std::vector<double>(num_class, 1.0));
    for (int i = 0; i < num_class; ++i) auc_mu_weights_matrix[i][i] = 0.0;
  } else {
    if (auc_mu_weights.size() != static_cast<size_t>(num_class * num_class)) {
      Log::Fatal("auc_mu_weights must have %d elements, but found %zu", num_class * num_class, auc_mu_weights.size());
    }
    auc_mu_weights_matrix.assign(num_class, std::vector<double>(num_class, 0.0));
    for (int i = 0; i < num_class; ++i)
      for (int j = 0; j < num_class; ++j)
        auc_mu_weights_matrix[i][j] = (i == j) ? 0.0 : auc_mu_weights[i * num_class + j];
  }
  interaction_constraints_vector = interaction_constraints.empty()
                                       ? std::vector<std::vector<int>>()
                                       : ParseArrayOfArrays(interaction_constraints);
  std::sort(eval_at.begin(), eval_at.end());
  {
    std::vector<std::string> nv;
    for (auto& s : valid) {
      if (s != data) nv.push_back(s);
      else is_provide_training_metric = true;
    }
    valid = nv;
  }
  if (task == "save_binary") save_binary = true;
  static const std::set<std::string> kTargets = {
      "ndcg", "lambdaloss-ndcg", "lambdaloss-ndcg-plus-plus", "bndcg", "lambdaloss-bndcg",
      "lambdaloss-bndcg-plus-plus", "precision", "arpk", "lambdaloss-arp1", "lambdaloss-arp2",
      "ranknet", "bin-ranknet", "lambdagap-s", "lambdagap-x", "lambdagap-s-plus", "lambdagap-x-plus",
      "lambdagap-s-plus-plus", "lambdagap-x-plus-plus"};
  lambdarank_target = common::ToLower(lambdarank_target);
  if (kTargets.count(lambdarank_target) == 0) {
    Log::Fatal("Unknown lambdarank_target %s", lambdarank_target.c_str());
  }
  CheckParamConflict(params);
}

void Config::CheckParamConflict(const ParamMap& params) {
  auto is_multi = [](const std::string& o) { return o == "multiclass" || o == "multiclassova"; };
  const bool custom = objective == "custom" || objective == "none" || objective == "null" || objective == "na";
  bool obj_multi = is_multi(objective) || (custom && num_class > 1);
  if (obj_multi) {
    if (num_class <= 1) Log::Fatal("Number of classes should be specified and greater than 1 for multiclass training");
  } else if (task == "train" && num_class != 1) {
    Log::Fatal("Number of classes must be 1 for non-multiclass training");
  }
  for (auto& m : metric) {
    bool mm = is_multi(m) || m == "multi_logloss" || m == "multi_error" || m == "auc_mu" ||
              (m == "custom" && num_class > 1);
    if (obj_multi != mm) Log::Fatal("Multiclass objective and metrics don't match");
  }
  if (num_machines > 1) {
    is_parallel = true;
  } else {
    is_parallel = false;
    tree_learner = "serial";
  }
  if (tree_learner == "serial") {
    is_parallel = false;
    num_machines = 1;
  }
  is_data_based_parallel = (tree_learner == "data" || tree_learner == "voting");
  if (is_data_based_parallel && tree_learner == "data" && histogram_pool_size >= 0) histogram_pool_size = -1;
  if (is_data_based_parallel && !forcedsplits_filename.empty()) {
    Log::Fatal("Don't support forcedsplits in %s tree learner", tree_learner.c_str());
  }
  if (max_depth > 0 && (params.count("num_leaves") == 0 || params.at("num_leaves").empty())) {
    double full = std::pow(2.0, max_depth);
    if (full < num_leaves) num_leaves = static_cast<int>(full);
  }
  if (linear_tree) {
    if (tree_learner != "serial") {
      tree_learner = "serial";
      Log::Warning("Linear tree learner must be serial.");
    }
    if (zero_as_missing) Log::Fatal("zero_as_missing must be false when fitting linear trees.");
    if (objective == "regression_l1") Log::Fatal("Cannot use regression_l1 objective when fitting linear trees.");
  }
  if (path_smooth > kEpsilon && min_data_in_leaf < 2) {
    min_data_in_leaf = 2;
    Log::Warning("min_data_in_leaf has been increased to 2 because this is required when path smoothing is active.");
  }
  if (is_parallel && (monotone_constraints_method == "intermediate" || monotone_constraints_method == "advanced")) {
    monotone_constraints_method = "basic";
  }
  if (feature_fraction_bynode != 1.0 &&
      (monotone_constraints_method == "intermediate" || monotone_constraints_method == "advanced")) {
    monotone_constraints_method = "basic";
  }
  if (min_data_in_leaf <= 0 && min_sum_hessian_in_leaf <= kEpsilon) {
    Log::Warning("Cannot set both min_data_in_leaf and min_sum_hessian_in_leaf to 0. Will set min_data_in_leaf to 1.");
    min_data_in_leaf = 1;
  }
  if (boosting == "goss") {
    boosting = "gbdt";
    data_sample_strategy = "goss";
  }
  if (bagging_by_query && data_sample_strategy != "bagging") bagging_by_query = false;
}

std::string Config::ToString() const {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss.precision(17);
  ss << "[boosting: " << boosting << "]\n";
  ss << "[objective: " << objective << "]\n";
  ss << "[metric: " << common::Join(metric, ",") << "]\n";
  ss << "[tree_learner: " << tree_learner << "]\n";
  ss << "[device_type: " << device_type << "]\n";
  auto vec_int8 = [](const std::vector<int8_t>& v) {
    std::vector<int> t(v.begin(), v.end());
    return common::Join(t, ",");
  };
#define LGAP_SAVE_STR(name) ss << "[" #name ": " << name << "]\n";
#define LGAP_SAVE_INT(name) ss << "[" #name ": " << name << "]\n";
#define LGAP_SAVE_DBL(name) ss << "[" #name ": " << common::FormatG(name) << "]\n";
#define LGAP_SAVE_BOOL(name) ss << "[" #name ": " << (name ? 1 : 0) << "]\n";
#define LGAP_SAVE_VSTR(name) ss << "[" #name ": " << common::Join(name, ",") << "]\n";
#define LGAP_SAVE_VINT(name) ss << "[" #name ": " << common::Join(name, ",") << "]\n";
#define LGAP_SAVE_VDBL(name) ss << "[" #name ": " << common::Join(name, ",") << "]\n";
#define LGAP_SAVE_VI8(name) ss << "[" #name ": " << vec_int8(name) << "]\n";
#define LGAP_SAVE_VI32(name) ss << "[" #name ": " << common::Join(name, ",") << "]\n";
#define LGAP_PARAM(kind, name, def, aliases, save, check) \
  if (save) { LGAP_SAVE_##kind(name) }
#include "lgap/config_params.def"
#undef LGAP_PARAM
  std::string out = ss.str();
  // the five leading keys above are also flagged save in the table for some; dedupe data_sample_strategy
  return out;
}

std::string Config::DumpAliases() {
  std::stringstream ss;
  ss << "{\n";
  bool first = true;
  for (auto& p : ParamTable()) {
    ss << (first ? "   \"" : "   , \"") << p.name << "\": [";
    first = false;
    auto al = common::Split(p.aliases, ',');
    for (size_t i = 0; i < al.size(); ++i) ss << (i ? ", " : "") << "\"" << al[i] << "\"";
    ss << "]\n";
  }
  ss << "}\n";
  return ss.str();
}

std::string Config::ParameterKind(const std::string& name) {
  for (auto& p : ParamTable()) {
    if (name == p.name) return p.kind;
  }
  return "";
}

std::string Config::DumpParameterTypes() {
  std::stringstream ss;
  ss << "{";
  bool first = true;
  for (auto& p : ParamTable()) {
    std::string k = p.kind;
    std::string t = k == "STR" ? "string" : k == "INT" ? "int" : k == "DBL" ? "double" : k == "BOOL" ? "bool"
                  : k == "VSTR" ? "vector<string>" : k == "VDBL" ? "vector<double>" : "vector<int>";
    ss << (first ? "" : ",") << "\"" << p.name << "\":\"" << t << "\"";
    first = false;
  }
  ss << "}";
  return ss.str();
}

}  // namespace lgap
