// Text data loading: CSV / TSV / LibSVM auto-detection (reference
// src/io/parser.cpp:179-317), label / weight / group / ignore columns with the
// reference's index conventions, side files, and rank partitioning for
// distributed training (dataset_loader.cpp:962-1001).
#include <omp.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <set>
#include <sstream>
#include <unordered_map>

#include "lgap/omp_errors.h"
#include "lgap/common.h"
#include "lgap/dataset.h"
#include "lgap/log.h"
#include "lgap/random.h"

#include "lgap/parser.h"

namespace lgap {

namespace {

enum class TextFormat { CSV, TSV, LIBSVM, INVALID };

std::vector<std::string> ReadAllLines(const std::string& filename) {
  std::ifstream in(filename, std::ios::binary);
  if (!in) Log::Fatal("Data file %s doesn't exist.", filename.c_str());
  std::string text((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  std::vector<std::string> lines;
  size_t s = 0;
  for (size_t i = 0; i <= text.size(); ++i) {
    if (i == text.size() || text[i] == '\n') {
      size_t e = i;
      if (e > s && text[e - 1] == '\r') --e;
      if (e > s) lines.emplace_back(text.data() + s, e - s);
      s = i + 1;
    }
  }
  return lines;
}

void Stat(const std::string& l, int* comma, int* tab, int* colon) {
  *comma = *tab = *colon = 0;
  for (char c : l) {
    if (c == ',') ++*comma;
    else if (c == '\t') ++*tab;
    else if (c == ':') ++*colon;
  }
}

TextFormat Detect(const std::vector<std::string>& lines, size_t first) {
  if (lines.size() <= first) return TextFormat::INVALID;
  int c1, t1, k1;
  Stat(lines[first], &c1, &t1, &k1);
  if (lines.size() == first + 1) {
    if (k1 > 0) return TextFormat::LIBSVM;
    if (t1 > 0) return TextFormat::TSV;
    if (c1 > 0) return TextFormat::CSV;
    return TextFormat::TSV;  // single column: treat as tsv
  }
  int c2, t2, k2;
  Stat(lines[first + 1], &c2, &t2, &k2);
  if (k1 > 0 || k2 > 0) return TextFormat::LIBSVM;
  if (t1 == t2 && t1 > 0) return TextFormat::TSV;
  if (c1 == c2 && c1 > 0) return TextFormat::CSV;
  if (t1 == 0 && c1 == 0) return TextFormat::TSV;
  return TextFormat::INVALID;
}

int ResolveColumn(const std::string& spec, const std::vector<std::string>& names, bool allow_missing = true) {
  if (spec.empty()) return -1;
  if (common::StartsWith(spec, "name:")) {
    std::string n = spec.substr(5);
    for (size_t i = 0; i < names.size(); ++i) if (names[i] == n) return static_cast<int>(i);
    if (!allow_missing) Log::Fatal("Could not find column %s in data file", n.c_str());
    return -1;
  }
  return common::AtoiOrDie(spec);
}

std::vector<int> ResolveColumnList(const std::string& spec, const std::vector<std::string>& names) {
  std::vector<int> out;
  if (spec.empty()) return out;
  if (common::StartsWith(spec, "name:")) {
    for (auto& n : common::Split(spec.substr(5), ',')) {
      for (size_t i = 0; i < names.size(); ++i) if (names[i] == n) out.push_back(static_cast<int>(i));
    }
    return out;
  }
  for (auto& t : common::Split(spec, ',')) out.push_back(common::AtoiOrDie(t));
  return out;
}

// One text line -> (feature row, label, weight, group id). Feature indices have
// the label column removed (CSV/TSV) or are taken as written (LibSVM).
void ParseLine(const std::string& line, TextFormat fmt, char delim, int label_idx, int weight_idx, int group_idx,
               std::vector<std::pair<int, double>>* row, float* label, float* weight, double* gid, int* maxcol) {
  row->clear();
  if (fmt == TextFormat::LIBSVM) {
    const char* p = line.c_str();
    // optional leading label (a token without ':')
    while (*p == ' ' || *p == '\t') ++p;
    const char* q = p;
    while (*q && *q != ' ' && *q != '\t' && *q != ':') ++q;
    if (*q != ':' && label_idx >= 0) {
      double v;
      common::Atof(p, &v);
      *label = static_cast<float>(v);
      p = q;
    }
    while (*p) {
      while (*p == ' ' || *p == '\t') ++p;
      if (!*p) break;
      char* e;
      long idx = std::strtol(p, &e, 10);
      if (*e != ':') break;
      double v;
      p = common::Atof(e + 1, &v);
      if (idx == weight_idx) *weight = static_cast<float>(v);
      if (idx == group_idx) *gid = v;
      if (std::isnan(v) || std::fabs(v) > kZeroThreshold) row->emplace_back(static_cast<int>(idx), v);
      if (idx > *maxcol) *maxcol = static_cast<int>(idx);
    }
    return;
  }
  const char* p = line.c_str();
  int col = 0;   // raw column index
  int fcol = 0;  // feature column index (label removed)
  while (true) {
    double v;
    const char* e = common::Atof(p, &v);
    if (col == label_idx) {
      *label = static_cast<float>(v);
    } else {
      if (fcol == weight_idx) *weight = static_cast<float>(v);
      if (fcol == group_idx) *gid = v;
      if (std::isnan(v) || std::fabs(v) > kZeroThreshold) row->emplace_back(fcol, v);
      ++fcol;
    }
    ++col;
    while (*e && *e != delim) ++e;
    if (!*e) break;
    p = e + 1;
  }
  if (fcol - 1 > *maxcol) *maxcol = fcol - 1;
}

}  // namespace

void ParseTextFile(const std::string& filename, bool header, int label_idx, OwnedSparseSource* rows,
                   std::vector<float>* labels, std::vector<std::string>* header_names, int* out_label_idx,
                   const std::vector<int>& ignore_cols, int weight_idx, std::vector<float>* weights, int group_idx,
                   std::vector<double>* group_ids) {
  auto lines = ReadAllLines(filename);
  size_t first = 0;
  if (header && !lines.empty()) {
    first = 1;
    if (header_names) {
      int c, t, k;
      Stat(lines[0], &c, &t, &k);
      *header_names = common::SplitAny(lines[0], t > 0 ? "\t" : (c > 0 ? "," : " "));
      for (auto& n : *header_names) n = common::Trim(n);
    }
  }
  TextFormat fmt = Detect(lines, first);
  // a binary Dataset file is not text (reference parser.cpp:265 on the same input)
  const bool binary = first < lines.size() && lines[first].rfind("______LambdaGap_Binary_File_Token______", 0) == 0;
  if (fmt == TextFormat::INVALID || binary) {
    Log::Fatal("Unknown format of training data. Only CSV, TSV, and LibSVM (zero-based) formatted text files are supported.");
  }
  const size_t n = lines.size() - first;
  rows->rows.assign(n, {});
  labels->assign(n, 0.0f);
  if (weights && weight_idx >= 0) weights->assign(n, 1.0f);
  if (group_ids && group_idx >= 0) group_ids->assign(n, 0.0);
  std::vector<int> maxcol(omp_get_max_threads(), -1);
  const char delim = fmt == TextFormat::CSV ? ',' : '\t';
  if (out_label_idx) *out_label_idx = label_idx;
  OmpErrors errs;  // a malformed line raises from ParseLine inside the region
#pragma omp parallel for schedule(static, 1024)
  for (size_t r = 0; r < n; ++r) {
    errs.Run([&] {
      const int tid = omp_get_thread_num();
      float w = 1.0f;
      double gid = 0.0;
      ParseLine(lines[first + r], fmt, delim, label_idx, weight_idx, group_idx, &rows->rows[r], &(*labels)[r], &w,
                &gid, &maxcol[tid]);
      if (weights && weight_idx >= 0) (*weights)[r] = w;
      if (group_ids && group_idx >= 0) (*group_ids)[r] = gid;
    });
  }
  errs.Rethrow();
  int mc = -1;
  for (int m : maxcol) mc = std::max(mc, m);
  rows->ncol = mc + 1;

  // drop ignored / weight / group columns from the feature values (they remain in the index space)
  std::set<int> drop(ignore_cols.begin(), ignore_cols.end());
  if (weight_idx >= 0) drop.insert(weight_idx);
  if (group_idx >= 0) drop.insert(group_idx);
  if (!drop.empty()) {
#pragma omp parallel for schedule(static, 1024)
    for (size_t r = 0; r < n; ++r) {
      auto& row = rows->rows[r];
      row.erase(std::remove_if(row.begin(), row.end(), [&](const std::pair<int, double>& kv) { return drop.count(kv.first) > 0; }),
                row.end());
    }
  }
}

// Two-round loading (reference dataset_loader.cpp two_round / TextReader sampling):
// pass 1 streams the file once to count rows, reservoir-sample
// bin_construct_sample_cnt lines for the bin mappers and decide rank membership;
// pass 2 streams it again and packs rows chunk by chunk, so the parsed text is
// never resident as a whole (long-data analogue of the reference's design).
namespace {
struct TwoRoundSpec {
  int label_idx, weight_idx, group_idx;
  std::vector<std::string> feat_names;
  std::vector<int> cats;
  Config c2;
};

bool NextDataLine(std::istream& in, std::string* line) {
  while (std::getline(in, *line)) {
    if (!line->empty() && line->back() == '\r') line->pop_back();
    if (!line->empty()) return true;
  }
  return false;
}

std::unique_ptr<Dataset> LoadTwoRound(const std::string& filename, const Config& cfg, const Dataset* reference,
                                      int rank, int num_machines, const TwoRoundSpec& sp) {
  std::ifstream in(filename, std::ios::binary);
  if (!in) Log::Fatal("Data file %s doesn't exist.", filename.c_str());
  std::string line;
  if (cfg.header) NextDataLine(in, &line);
  std::vector<std::string> head, sample;
  std::vector<double> gids_all;
  const size_t want = static_cast<size_t>(std::max(1, cfg.bin_construct_sample_cnt));
  Random sampler(cfg.data_random_seed);
  size_t n = 0;
  TextFormat fmt = TextFormat::INVALID;
  char delim = '\t';
  int maxcol = -1;
  while (NextDataLine(in, &line)) {
    if (head.size() < 2) {
      head.push_back(line);
      if (head.size() == 2) {
        fmt = Detect(head, 0);
        delim = fmt == TextFormat::CSV ? ',' : '\t';
      }
    }
    if (!reference) {
      if (sample.size() < want) {
        sample.push_back(line);
      } else {
        const size_t j = static_cast<size_t>(sampler.NextInt(0, static_cast<int>(std::min<size_t>(n + 1, 0x7fffffff))));
        if (j < want) sample[j] = line;
      }
    }
    if (sp.group_idx >= 0) {
      std::vector<std::pair<int, double>> row;
      float lab = 0.f, w = 1.f;
      double g = 0.0;
      if (fmt == TextFormat::INVALID) fmt = Detect(head, 0), delim = fmt == TextFormat::CSV ? ',' : '\t';
      ParseLine(line, fmt, delim, sp.label_idx, sp.weight_idx, sp.group_idx, &row, &lab, &w, &g, &maxcol);
      gids_all.push_back(g);
    }
    ++n;
  }
  if (fmt == TextFormat::INVALID) fmt = Detect(head, 0), delim = fmt == TextFormat::CSV ? ',' : '\t';
  if (fmt == TextFormat::INVALID) Log::Fatal("Unknown format of training data %s", filename.c_str());
  // rank membership, drawn in the one-round loader's order (rows, or whole queries)
  std::vector<char> keep(n, 1);
  std::vector<data_size_t> qb;
  if (sp.group_idx >= 0) {
    qb.push_back(0);
    for (size_t i = 1; i < n; ++i) if (gids_all[i] != gids_all[i - 1]) qb.push_back(static_cast<data_size_t>(i));
    qb.push_back(static_cast<data_size_t>(n));
  }
  if (num_machines > 1 && !cfg.pre_partition) {
    Random rnd(cfg.data_random_seed);
    if (!qb.empty()) {
      std::vector<data_size_t> nqb = {0};
      for (size_t q = 0; q + 1 < qb.size(); ++q) {
        const bool mine = rnd.NextShort(0, num_machines) == rank;
        for (data_size_t i = qb[q]; i < qb[q + 1]; ++i) keep[i] = mine;
        if (mine) nqb.push_back(nqb.back() + (qb[q + 1] - qb[q]));
      }
      qb = nqb;
    } else {
      for (size_t i = 0; i < n; ++i) keep[i] = rnd.NextShort(0, num_machines) == rank;
    }
  }
  data_size_t n_local = 0;
  for (char k : keep) n_local += k;
  // bin mappers (and bundles) from the sample, or the reference's
  auto ds = std::make_unique<Dataset>();
  if (reference) {
    ds->InitEmptyLike(*reference, n_local);
  } else {
    OwnedSparseSource srows;
    srows.rows.resize(sample.size());
    int smax = -1;
    for (size_t r = 0; r < sample.size(); ++r) {
      float lab, w;
      double g;
      ParseLine(sample[r], fmt, delim, sp.label_idx, sp.weight_idx, sp.group_idx, &srows.rows[r], &lab, &w, &g, &smax);
    }
    srows.ncol = std::max(smax, maxcol) + 1;
    Dataset ref;
    ref.Construct(srows, sp.c2, nullptr, sp.feat_names, sp.cats);
    ds->InitEmptyLike(ref, n_local);
  }
  sample.clear();
  sample.shrink_to_fit();
  // pass 2: parse and pack in chunks
  in.clear();
  in.seekg(0);
  if (cfg.header) NextDataLine(in, &line);
  constexpr size_t kChunk = 1 << 16;
  std::vector<std::string> lines;
  lines.reserve(kChunk);
  std::vector<float> labels(n_local), weights(sp.weight_idx >= 0 ? n_local : 0);
  data_size_t filled = 0;
  size_t row_id = 0;
  auto flush = [&]() {
    OwnedSparseSource chunk;
    chunk.ncol = ds->num_total_features();
    chunk.rows.resize(lines.size());
    std::vector<int> mc(omp_get_max_threads(), -1);
    OmpErrors errs;
#pragma omp parallel for schedule(static, 256)
    for (size_t r = 0; r < lines.size(); ++r) {
      errs.Run([&] {
        float w = 1.0f;
        double g = 0.0;
        ParseLine(lines[r], fmt, delim, sp.label_idx, sp.weight_idx, sp.group_idx, &chunk.rows[r],
                  &labels[filled + r], &w, &g, &mc[omp_get_thread_num()]);
        if (sp.weight_idx >= 0) weights[filled + r] = w;
        // weight / group columns are not features
        if (sp.weight_idx >= 0 || sp.group_idx >= 0) {
          auto& row = chunk.rows[r];
          row.erase(std::remove_if(row.begin(), row.end(),
                                   [&](const std::pair<int, double>& kv) {
                                     return kv.first == sp.weight_idx || kv.first == sp.group_idx;
                                   }),
                    row.end());
        }
      });
    }
    errs.Rethrow();
    ds->PushRows(chunk, filled);
    filled += static_cast<data_size_t>(lines.size());
    lines.clear();
  };
  while (NextDataLine(in, &line)) {
    if (keep[row_id++]) {
      lines.push_back(line);
      if (lines.size() == kChunk) flush();
    }
  }
  if (!lines.empty()) flush();
  ds->metadata().SetLabel(labels.data(), n_local);
  if (sp.weight_idx >= 0) ds->metadata().SetWeights(weights.data(), n_local);
  if (!qb.empty()) ds->metadata().SetQueryBoundaries(qb);
  if (num_machines <= 1 || cfg.pre_partition) ds->metadata().LoadSideFiles(filename);
  Log::Info("Loaded %d rows x %d features from %s (two-round)", n_local, ds->num_total_features(), filename.c_str());
  return ds;
}
}  // namespace

std::unique_ptr<Dataset> LoadDatasetFromFile(const std::string& filename, const Config& cfg, const Dataset* reference,
                                             int rank, int num_machines) {
  if (Dataset::IsBinaryFile(filename)) {
    Log::Info("Loading binary dataset %s", filename.c_str());
    return Dataset::LoadBinary(filename);
  }
  if (Dataset::IsBinaryFile(filename + ".bin")) {
    Log::Info("Loading binary dataset %s.bin", filename.c_str());
    return Dataset::LoadBinary(filename + ".bin");
  }
  std::vector<std::string> names;
  if (cfg.header) {
    std::ifstream in(filename);
    std::string l;
    std::getline(in, l);
    if (!l.empty() && l.back() == '\r') l.pop_back();
    int c, t, k;
    Stat(l, &c, &t, &k);
    names = common::SplitAny(l, t > 0 ? "\t" : (c > 0 ? "," : " "));
    for (auto& s : names) s = common::Trim(s);
  }
  int label_idx = 0;
  if (!cfg.label_column.empty()) label_idx = ResolveColumn(cfg.label_column, names, false);
  std::vector<std::string> feat_names;
  for (size_t i = 0; i < names.size(); ++i) if (static_cast<int>(i) != label_idx) feat_names.push_back(names[i]);
  // weight / group / ignore indices are relative to feature columns (label removed), except name: specs
  auto rel = [&](int raw) { return raw; };
  int weight_idx = -1, group_idx = -1;
  if (!cfg.weight_column.empty()) {
    weight_idx = common::StartsWith(cfg.weight_column, "name:") ? ResolveColumn(cfg.weight_column, feat_names)
                                                                : rel(common::AtoiOrDie(cfg.weight_column));
  }
  if (!cfg.group_column.empty()) {
    group_idx = common::StartsWith(cfg.group_column, "name:") ? ResolveColumn(cfg.group_column, feat_names)
                                                              : rel(common::AtoiOrDie(cfg.group_column));
  }
  std::vector<int> ignore = common::StartsWith(cfg.ignore_column, "name:")
                                ? ResolveColumnList(cfg.ignore_column, feat_names)
                                : ResolveColumnList(cfg.ignore_column, {});
  if (cfg.two_round && cfg.parser_config_file.empty()) {
    TwoRoundSpec sp;
    sp.label_idx = label_idx;
    sp.weight_idx = weight_idx;
    sp.group_idx = group_idx;
    sp.feat_names = reference ? std::vector<std::string>() : feat_names;
    if (!cfg.categorical_feature.empty()) {
      sp.cats = common::StartsWith(cfg.categorical_feature, "name:")
                    ? ResolveColumnList(cfg.categorical_feature, feat_names)
                    : ResolveColumnList(cfg.categorical_feature, {});
    }
    sp.c2 = cfg;
    std::string ig;
    for (size_t i = 0; i < ignore.size(); ++i) ig += (i ? "," : "") + std::to_string(ignore[i]);
    if (weight_idx >= 0) ig += (ig.empty() ? "" : ",") + std::to_string(weight_idx);
    if (group_idx >= 0) ig += (ig.empty() ? "" : ",") + std::to_string(group_idx);
    sp.c2.ignore_column = ig;
    auto ds = LoadTwoRound(filename, cfg, reference, rank, num_machines, sp);
    if (cfg.save_binary) ds->SaveBinary(filename + ".bin");
    return ds;
  }
  OwnedSparseSource rows;
  std::vector<float> labels, weights;
  std::vector<double> gids;
  // custom parser plugin (parser_config_file): every line through the registered class
  const std::string parser_cfg = cfg.parser_config_file.empty()
                                     ? std::string()
                                     : GenerateParserConfigStr(filename, cfg.parser_config_file, cfg.header, label_idx);
  if (!parser_cfg.empty()) {
    auto parser = CreateCustomParser(parser_cfg);
    auto lines = ReadAllLines(filename);
    const size_t first = cfg.header && !lines.empty() ? 1 : 0;
    const size_t nl = lines.size() - first;
    rows.rows.assign(nl, {});
    labels.assign(nl, 0.0f);
    std::vector<int> maxcol(omp_get_max_threads(), -1);
    OmpErrors errs;
#pragma omp parallel for schedule(static, 1024)
    for (size_t r = 0; r < nl; ++r) {
      errs.Run([&] {
        double lab = 0.0;
        parser->ParseOneLine(lines[first + r].c_str(), &rows.rows[r], &lab);
        labels[r] = static_cast<float>(lab);
        int& m = maxcol[omp_get_thread_num()];
        for (const auto& kv : rows.rows[r]) m = std::max(m, kv.first);
      });
    }
    errs.Rethrow();
    int mc = std::max(-1, parser->NumFeatures() - 1);
    for (int m : maxcol) mc = std::max(mc, m);
    rows.ncol = mc + 1;
    weight_idx = group_idx = -1;
  } else {
    ParseTextFile(filename, cfg.header, label_idx, &rows, &labels, nullptr, nullptr, ignore, weight_idx, &weights,
                  group_idx, &gids);
  }
  if (reference) rows.ncol = std::max(rows.ncol, reference->num_total_features());
  data_size_t n = static_cast<data_size_t>(rows.rows.size());

  // query boundaries from a group column (consecutive equal ids)
  std::vector<data_size_t> qb;
  if (group_idx >= 0) {
    qb.push_back(0);
    for (data_size_t i = 1; i < n; ++i) if (gids[i] != gids[i - 1]) qb.push_back(i);
    qb.push_back(n);
  }
  // distributed: random partition of rows (or whole queries) across ranks
  std::vector<data_size_t> used;
  if (num_machines > 1 && !cfg.pre_partition) {
    Random rnd(cfg.data_random_seed);
    if (!qb.empty()) {
      std::vector<data_size_t> nqb = {0};
      for (size_t q = 0; q + 1 < qb.size(); ++q) {
        if (rnd.NextShort(0, num_machines) == rank) {
          for (data_size_t i = qb[q]; i < qb[q + 1]; ++i) used.push_back(i);
          nqb.push_back(static_cast<data_size_t>(used.size()));
        }
      }
      qb = nqb;
    } else {
      for (data_size_t i = 0; i < n; ++i) if (rnd.NextShort(0, num_machines) == rank) used.push_back(i);
    }
    OwnedSparseSource part;
    part.ncol = rows.ncol;
    std::vector<float> pl, pw;
    for (auto i : used) {
      part.rows.push_back(std::move(rows.rows[i]));
      pl.push_back(labels[i]);
      if (!weights.empty()) pw.push_back(weights[i]);
    }
    rows = std::move(part);
    labels = pl;
    weights = pw;
    n = static_cast<data_size_t>(rows.rows.size());
  }
  std::vector<int> cats;
  if (!cfg.categorical_feature.empty()) {
    cats = common::StartsWith(cfg.categorical_feature, "name:") ? ResolveColumnList(cfg.categorical_feature, feat_names)
                                                                : ResolveColumnList(cfg.categorical_feature, {});
  }
  Config c2 = cfg;
  {
    std::string ig;
    for (size_t i = 0; i < ignore.size(); ++i) ig += (i ? "," : "") + std::to_string(ignore[i]);
    if (weight_idx >= 0) ig += (ig.empty() ? "" : ",") + std::to_string(weight_idx);
    if (group_idx >= 0) ig += (ig.empty() ? "" : ",") + std::to_string(group_idx);
    c2.ignore_column = ig;
  }
  auto ds = std::make_unique<Dataset>();
  // a custom parser defines its own column layout: the raw header's names would not line up
  // with it, so its features take the default Column_i names (reference dataset_loader.cpp:86-89)
  const bool header_names = !reference && parser_cfg.empty();
  ds->Construct(rows, c2, reference, header_names ? feat_names : std::vector<std::string>(), cats);
  ds->metadata().SetLabel(labels.data(), n);
  if (weight_idx >= 0) ds->metadata().SetWeights(weights.data(), n);
  if (!qb.empty()) ds->metadata().SetQueryBoundaries(qb);
  if (num_machines <= 1 || cfg.pre_partition) ds->metadata().LoadSideFiles(filename);
  ds->set_parser_config(parser_cfg);
  Log::Info("Loaded %d rows x %d features from %s", n, ds->num_total_features(), filename.c_str());
  if (cfg.save_binary) ds->SaveBinary(filename + ".bin");
  return ds;
}

}  // namespace lgap
