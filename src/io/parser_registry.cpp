// Custom parser registry (include/lgap/parser.h). Reference: src/io/parser.cpp:287-318,
// include/LightGBM/dataset.h:463-486.
#include "lgap/parser.h"

#include <cstdlib>
#include <fstream>
#include <sstream>

#include "lgap/log.h"

namespace lgap {

ParserFactory& ParserFactory::Instance() {
  static ParserFactory f;
  return f;
}

void ParserFactory::Register(const std::string& class_name, std::function<Parser*(const std::string&)> make) {
  makers_[class_name] = std::move(make);
}

std::unique_ptr<Parser> ParserFactory::Create(const std::string& class_name, const std::string& config) const {
  auto it = makers_.find(class_name);
  if (it == makers_.end()) return nullptr;
  return std::unique_ptr<Parser>(it->second(config));
}

namespace {
// position of the value of "key" in a flat JSON object, npos if absent
size_t FindValue(const std::string& s, const std::string& key, size_t* end) {
  const std::string q = "\"" + key + "\"";
  size_t p = s.find(q);
  while (p != std::string::npos) {
    size_t c = p + q.size();
    while (c < s.size() && (s[c] == ' ' || s[c] == '\t' || s[c] == '\n' || s[c] == '\r')) ++c;
    if (c < s.size() && s[c] == ':') {
      ++c;
      while (c < s.size() && (s[c] == ' ' || s[c] == '\t' || s[c] == '\n' || s[c] == '\r')) ++c;
      size_t e = c;
      if (e < s.size() && s[e] == '"') {
        ++e;
        while (e < s.size() && s[e] != '"') e += (s[e] == '\\' && e + 1 < s.size()) ? 2 : 1;
        *end = e + 1;
      } else {
        while (e < s.size() && s[e] != ',' && s[e] != '}') ++e;
        *end = e;
      }
      return c;
    }
    p = s.find(q, p + 1);
  }
  return std::string::npos;
}
}  // namespace

std::string GetFromParserConfig(const std::string& config, const std::string& key) {
  size_t end = 0;
  const size_t b = FindValue(config, key, &end);
  if (b == std::string::npos) return "";
  std::string v = config.substr(b, end - b);
  while (!v.empty() && (v.back() == ' ' || v.back() == '\n' || v.back() == '\r' || v.back() == '\t')) v.pop_back();
  if (v.size() >= 2 && v.front() == '"' && v.back() == '"') v = v.substr(1, v.size() - 2);
  return v;
}

std::string SaveToParserConfig(const std::string& config, const std::string& key, const std::string& value) {
  std::string esc;
  for (char ch : value) {
    if (ch == '"' || ch == '\\') esc += '\\';
    esc += ch;
  }
  size_t end = 0;
  const size_t b = FindValue(config, key, &end);
  if (b != std::string::npos) return config.substr(0, b) + "\"" + esc + "\"" + config.substr(end);
  const size_t close = config.rfind('}');
  if (close == std::string::npos) Log::Fatal("Malformed parser config (expected a JSON object): %s", config.c_str());
  size_t last = close;
  while (last > 0 && (config[last - 1] == ' ' || config[last - 1] == '\n' || config[last - 1] == '\r' || config[last - 1] == '\t')) --last;
  const bool empty = last > 0 && config[last - 1] == '{';
  return config.substr(0, last) + (empty ? "" : ", ") + "\"" + key + "\": \"" + esc + "\"" + config.substr(last);
}

std::string GenerateParserConfigStr(const std::string& data_file, const std::string& config_file, bool header,
                                    int label_idx) {
  std::ifstream in(config_file);
  if (!in) Log::Fatal("Cannot open parser config file %s", config_file.c_str());
  std::stringstream ss;
  ss << in.rdbuf();
  std::string cfg = ss.str();
  // the config is stored with the model: one line
  for (auto& ch : cfg) if (ch == '\n' || ch == '\r') ch = ' ';
  if (cfg.find_first_not_of(" \t") == std::string::npos) return "";
  if (header && GetFromParserConfig(cfg, "header").empty()) {
    std::ifstream d(data_file);
    std::string first;
    std::getline(d, first);
    if (!first.empty() && first.back() == '\r') first.pop_back();
    cfg = SaveToParserConfig(cfg, "header", first);
  }
  if (GetFromParserConfig(cfg, "labelId").empty()) cfg = SaveToParserConfig(cfg, "labelId", std::to_string(label_idx));
  return cfg;
}

std::unique_ptr<Parser> CreateCustomParser(const std::string& config) {
  const std::string cls = GetFromParserConfig(config, "className");
  Log::Info("Custom parser class name: %s", cls.c_str());
  auto p = ParserFactory::Instance().Create(cls, config);
  if (!p) Log::Fatal("Cannot find parser class '%s', please register first or check config format", cls.c_str());
  return p;
}

// ---------------------------------------------------------------------------
// Built-in plugin (also the worked example): delimited rows whose label is the LAST column,
// "delimiter" from the config (default ","). {"className": "lambdagap.label_last"}.
namespace {
class LabelLastParser : public Parser {
 public:
  explicit LabelLastParser(const std::string& config) {
    const std::string d = GetFromParserConfig(config, "delimiter");
    delim_ = d.empty() ? ',' : (d == "\\t" ? '\t' : d[0]);
  }
  void ParseOneLine(const char* str, std::vector<std::pair<int, double>>* out, double* label) const override {
    std::vector<double> vals;
    const char* p = str;
    while (*p) {
      char* e;
      const double v = std::strtod(p, &e);
      vals.push_back(e == p ? 0.0 : v);
      p = e;
      while (*p && *p != delim_) ++p;
      if (*p == delim_) ++p;
    }
    out->clear();
    if (vals.empty()) return;
    *label = vals.back();
    for (size_t i = 0; i + 1 < vals.size(); ++i) {
      if (vals[i] != 0.0) out->emplace_back(static_cast<int>(i), vals[i]);
    }
  }
  int NumFeatures() const override { return -1; }  // (the loader takes the widest row)

 private:
  char delim_ = ',';
};
const ParserReflector kLabelLast("lambdagap.label_last", [](const std::string& c) { return new LabelLastParser(c); });
}  // namespace

}  // namespace lgap
