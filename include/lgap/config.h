// Parameter struct generated from config_params.def (X-macro) plus the
// post-processing rules of the reference (src/io/config.cpp:99-512).
#pragma once

#include <string>
#include <unordered_map>
#include <vector>

#include "lgap/meta.h"

namespace lgap {

using ParamMap = std::unordered_map<std::string, std::string>;

struct Config {
#define LGAP_T_STR std::string
#define LGAP_T_INT int
#define LGAP_T_DBL double
#define LGAP_T_BOOL bool
#define LGAP_T_VSTR std::vector<std::string>
#define LGAP_T_VINT std::vector<int>
#define LGAP_T_VDBL std::vector<double>
#define LGAP_T_VI8 std::vector<int8_t>
#define LGAP_T_VI32 std::vector<int32_t>
#define LGAP_PARAM(kind, name, def, aliases, save, check) LGAP_T_##kind name = LGAP_T_##kind(def);
#include "lgap/config_params.def"
#undef LGAP_PARAM

  // derived
  bool is_parallel = false;
  bool is_data_based_parallel = false;
  std::vector<std::vector<double>> auc_mu_weights_matrix;
  std::vector<std::vector<int>> interaction_constraints_vector;

  Config() = default;
  explicit Config(const ParamMap& params) { Set(params); }

  void Set(const ParamMap& params);
  // "parameters:" section of a saved model (Config::ToString semantics)
  std::string ToString() const;
  bool IsDeviceLearner() const { return device_type == "gpu" || device_type == "cuda"; }

  // parsing helpers
  static ParamMap Str2Map(const char* parameters);
  static void KV2Map(std::unordered_map<std::string, std::vector<std::string>>* params, const char* kv);
  static void KeyAliasTransform(ParamMap* params);
  static std::string DumpAliases();
  static std::string DumpParameterTypes();
  static const std::unordered_map<std::string, std::string>& AliasTable();
  static bool IsKnownParameter(const std::string& name);
  // kind of a parameter in config_params.def (INT, DBL, BOOL, STR, VINT, ...), "" if unknown
  static std::string ParameterKind(const std::string& name);

 private:
  void GetMembersFromString(const ParamMap& params);
  void CheckParamConflict(const ParamMap& params);
};

std::string ParseObjectiveAlias(const std::string& type);
std::string ParseMetricAlias(const std::string& type);

}  // namespace lgap
