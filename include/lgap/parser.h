// Custom text parsers (`parser_config_file`). Reference: include/LightGBM/dataset.h:400-486
// (Parser / ParserFactory / ParserReflector) and src/io/parser.cpp:287-318.
//
// A plugin is a C++ class derived from lgap::Parser, linked into the process and registered
// by name with a static lgap::ParserReflector. A Dataset built from a text file with
// `parser_config_file` set reads the JSON config, looks the class up by its "className" and
// parses every line with it; the config string is stored in the model ("parser:" section) so
// predictions from files parse with the same class.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace lgap {

class Parser {
 public:
  Parser() = default;
  explicit Parser(const std::string& /*config*/) {}
  virtual ~Parser() = default;
  // one record (NUL-terminated) -> (feature column, value) pairs and the label (if present)
  virtual void ParseOneLine(const char* str, std::vector<std::pair<int, double>>* out_features,
                            double* out_label) const = 0;
  virtual int NumFeatures() const = 0;
};

class ParserFactory {
 public:
  static ParserFactory& Instance();
  void Register(const std::string& class_name, std::function<Parser*(const std::string&)> make);
  // nullptr when `class_name` is not registered
  std::unique_ptr<Parser> Create(const std::string& class_name, const std::string& config) const;

 private:
  std::map<std::string, std::function<Parser*(const std::string&)>> makers_;
};

// static registration: `static lgap::ParserReflector reg("MyParser", [](const std::string& c) {
//   return new MyParser(c); });`
class ParserReflector {
 public:
  ParserReflector(const std::string& class_name, std::function<Parser*(const std::string&)> make) {
    ParserFactory::Instance().Register(class_name, std::move(make));
  }
};

// flat JSON object helpers (reference common.h GetFromParserConfig / SaveToParserConfig)
std::string GetFromParserConfig(const std::string& config, const std::string& key);
std::string SaveToParserConfig(const std::string& config, const std::string& key, const std::string& value);
// the config file's text plus "header" (first line of a file with a header) and "labelId"
std::string GenerateParserConfigStr(const std::string& data_file, const std::string& config_file, bool header,
                                    int label_idx);
// the registered parser named by the config's "className" (fatal if none)
std::unique_ptr<Parser> CreateCustomParser(const std::string& config);

}  // namespace lgap
