// Labels, weights, init scores, query boundaries and positions
// (reference: src/io/metadata.cpp, side files :640,662).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <unordered_map>

#include "lgap/common.h"
#include "lgap/dataset.h"
#include "lgap/log.h"

namespace lgap {

void Metadata::Init(data_size_t num_data, int num_class_init_score) {
  num_data_ = num_data;
  label_.assign(num_data, 0.0f);
  weights_.clear();
  init_score_.clear();
  if (num_class_init_score > 0) init_score_.assign(static_cast<size_t>(num_data) * num_class_init_score, 0.0);
  query_boundaries_.clear();
  query_weights_.clear();
  positions_.clear();
}

void Metadata::SetLabel(const float* label, data_size_t len) {
  if (len != num_data_) Log::Fatal("Length of label is not same with #data");
  label_.assign(label, label + len);
  for (auto v : label_) {
    if (std::isnan(v) || std::isinf(v)) Log::Fatal("NaN or Inf found in label");
  }
}

void Metadata::SetRows(data_size_t start, data_size_t n, const float* label, const float* weight,
                       const double* init_score, const int32_t* query) {
  if (start < 0 || start + n > num_data_) Log::Fatal("Pushed metadata rows exceed the dataset size");
  if (label) std::copy(label, label + n, label_.begin() + start);
  if (weight) {
    if (weights_.empty()) weights_.assign(num_data_, 1.0f);
    std::copy(weight, weight + n, weights_.begin() + start);
  }
  if (init_score) {
    if (init_score_.empty()) init_score_.assign(num_data_, 0.0);
    std::copy(init_score, init_score + n, init_score_.begin() + start);
  }
  if (query) {
    if (pending_query_ids_.empty()) pending_query_ids_.assign(num_data_, -1);
    std::copy(query, query + n, pending_query_ids_.begin() + start);
  }
  if (start + n == num_data_) {
    if (!weights_.empty()) SetWeights(std::vector<float>(weights_).data(), num_data_);
    if (!pending_query_ids_.empty()) {
      // consecutive equal ids form one query
      std::vector<data_size_t> sizes;
      for (data_size_t i = 0; i < num_data_; ++i) {
        if (i == 0 || pending_query_ids_[i] != pending_query_ids_[i - 1]) sizes.push_back(0);
        ++sizes.back();
      }
      pending_query_ids_.clear();
      SetQuery(sizes.data(), static_cast<data_size_t>(sizes.size()));
    }
  }
}

void Metadata::SetWeights(const float* w, data_size_t len) {
  if (w == nullptr || len == 0) {
    weights_.clear();
    query_weights_.clear();
    return;
  }
  if (len != num_data_) Log::Fatal("Length of weights is not same with #data");
  weights_.assign(w, w + len);  // no sign check: the reference's SetWeights takes any value
  CalcQueryWeights();
}

void Metadata::SetInitScore(const double* s, size_t len) {
  if (s == nullptr || len == 0) {
    init_score_.clear();
    return;
  }
  if (len % static_cast<size_t>(num_data_) != 0) Log::Fatal("Initial score size doesn't match data size");
  init_score_.assign(s, s + len);
}

void Metadata::SetQuery(const data_size_t* sizes, data_size_t num_groups) {
  if (sizes == nullptr || num_groups == 0) {
    query_boundaries_.clear();
    query_weights_.clear();
    return;
  }
  std::vector<data_size_t> b(num_groups + 1, 0);
  for (data_size_t i = 0; i < num_groups; ++i) b[i + 1] = b[i] + sizes[i];
  if (b.back() != num_data_) Log::Fatal("Sum of query counts (%d) differs from the length of #data (%d)", b.back(), num_data_);
  query_boundaries_ = b;
  CalcQueryWeights();
}

void Metadata::SetQueryBoundaries(const std::vector<data_size_t>& b) {
  query_boundaries_ = b;
  CalcQueryWeights();
}

void Metadata::SetPosition(const int32_t* pos, data_size_t len) {
  if (pos == nullptr || len == 0) {
    positions_.clear();
    position_ids_.clear();
    return;
  }
  if (len != num_data_) Log::Fatal("Positions size (%d) doesn't match data size (%d)", len, num_data_);
  // remap arbitrary position values to dense ids 0..P-1 (keeps first-seen order sorted)
  std::vector<int32_t> uniq(pos, pos + len);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  std::unordered_map<int32_t, int32_t> id;
  position_ids_.clear();
  for (size_t i = 0; i < uniq.size(); ++i) {
    id[uniq[i]] = static_cast<int32_t>(i);
    position_ids_.push_back(std::to_string(uniq[i]));
  }
  positions_.resize(len);
  for (data_size_t i = 0; i < len; ++i) positions_[i] = id[pos[i]];
}

void Metadata::CalcQueryWeights() {
  query_weights_.clear();
  if (weights_.empty() || query_boundaries_.empty()) return;
  const data_size_t nq = num_queries();
  query_weights_.resize(nq);
  for (data_size_t q = 0; q < nq; ++q) {
    double s = 0.0;
    for (data_size_t i = query_boundaries_[q]; i < query_boundaries_[q + 1]; ++i) s += weights_[i];
    query_weights_[q] = static_cast<label_t>(s / (query_boundaries_[q + 1] - query_boundaries_[q]));
  }
}

void Metadata::Subset(const Metadata& src, const data_size_t* idx, data_size_t n) {
  num_data_ = n;
  label_.resize(n);
  for (data_size_t i = 0; i < n; ++i) label_[i] = src.label_[idx[i]];
  weights_.clear();
  if (!src.weights_.empty()) {
    weights_.resize(n);
    for (data_size_t i = 0; i < n; ++i) weights_[i] = src.weights_[idx[i]];
  }
  init_score_.clear();
  if (!src.init_score_.empty()) {
    size_t k = src.init_score_.size() / src.num_data_;
    init_score_.resize(k * n);
    for (size_t c = 0; c < k; ++c)
      for (data_size_t i = 0; i < n; ++i) init_score_[c * n + i] = src.init_score_[c * src.num_data_ + idx[i]];
  }
  positions_.clear();
  position_ids_ = src.position_ids_;
  if (!src.positions_.empty()) {
    positions_.resize(n);
    for (data_size_t i = 0; i < n; ++i) positions_[i] = src.positions_[idx[i]];
  }
  query_boundaries_.clear();
  query_weights_.clear();
  if (!src.query_boundaries_.empty()) {
    // keep whole queries only: idx must consist of complete, sorted queries
    std::vector<data_size_t> qof(src.num_data_);
    for (data_size_t q = 0; q < src.num_queries(); ++q)
      for (data_size_t i = src.query_boundaries_[q]; i < src.query_boundaries_[q + 1]; ++i) qof[i] = q;
    query_boundaries_.push_back(0);
    for (data_size_t i = 0; i < n; ++i) {
      if (i > 0 && qof[idx[i]] != qof[idx[i - 1]]) query_boundaries_.push_back(i);
    }
    query_boundaries_.push_back(n);
    if (n == 0) query_boundaries_ = {0};
    CalcQueryWeights();
  }
}

void Metadata::LoadSideFiles(const std::string& fn) {
  auto read_lines = [](const std::string& f) {
    std::vector<std::string> out;
    std::ifstream in(f);
    if (!in) return out;
    std::string line;
    while (std::getline(in, line)) {
      line = common::Trim(line);
      if (!line.empty()) out.push_back(line);
    }
    return out;
  };
  auto w = read_lines(fn + ".weight");
  if (!w.empty()) {
    std::vector<float> v;
    for (auto& s : w) v.push_back(static_cast<float>(common::AtofOrDie(s)));
    if (static_cast<data_size_t>(v.size()) == num_data_) {
      SetWeights(v.data(), num_data_);
      Log::Info("Loading weights...");
    }
  }
  auto q = read_lines(fn + ".query");
  if (q.empty()) q = read_lines(fn + ".group");
  if (!q.empty()) {
    std::vector<data_size_t> v;
    for (auto& s : q) v.push_back(common::AtoiOrDie(s));
    SetQuery(v.data(), static_cast<data_size_t>(v.size()));
    Log::Info("Loading query boundaries...");
  }
  auto init = read_lines(fn + ".init");
  if (!init.empty()) {
    std::vector<double> rows;
    size_t k = 0;
    for (auto& s : init) {
      auto vals = common::SplitAny(s, "\t ,");
      k = vals.size();
      for (auto& t : vals) rows.push_back(common::AtofOrDie(t));
    }
    // file is row-major [n x k]; internal layout is class-major
    std::vector<double> cm(rows.size());
    size_t n = rows.size() / std::max<size_t>(k, 1);
    for (size_t i = 0; i < n; ++i)
      for (size_t c = 0; c < k; ++c) cm[c * n + i] = rows[i * k + c];
    if (static_cast<data_size_t>(n) == num_data_) {
      init_score_ = cm;
      Log::Info("Loading initial scores...");
    }
  }
  auto pos = read_lines(fn + ".position");
  if (!pos.empty() && static_cast<data_size_t>(pos.size()) != num_data_) {
    // reference metadata.cpp:223-226 / 268-272
    Log::Fatal("Positions size (%d) doesn't match data size (%d)", static_cast<int>(pos.size()), num_data_);
  }
  if (!pos.empty()) {
    std::unordered_map<std::string, int32_t> id;
    position_ids_.clear();
    positions_.resize(num_data_);
    for (data_size_t i = 0; i < num_data_; ++i) {
      auto it = id.find(pos[i]);
      if (it == id.end()) {
        int32_t nid = static_cast<int32_t>(position_ids_.size());
        id[pos[i]] = nid;
        position_ids_.push_back(pos[i]);
        positions_[i] = nid;
      } else {
        positions_[i] = it->second;
      }
    }
  }
}

void Metadata::CheckOrPartition(data_size_t num_all, const std::vector<data_size_t>& used) {
  if (used.empty() || static_cast<data_size_t>(used.size()) == num_all) return;
  Metadata tmp = *this;
  Subset(tmp, used.data(), static_cast<data_size_t>(used.size()));
}

namespace {
template <typename T>
void PutVec(std::vector<char>* out, const std::vector<T>& v) {
  int64_t n = static_cast<int64_t>(v.size());
  out->insert(out->end(), reinterpret_cast<const char*>(&n), reinterpret_cast<const char*>(&n) + 8);
  out->insert(out->end(), reinterpret_cast<const char*>(v.data()), reinterpret_cast<const char*>(v.data() + v.size()));
}
template <typename T>
std::vector<T> GetVec(const char*& p) {
  int64_t n;
  std::memcpy(&n, p, 8);
  p += 8;
  std::vector<T> v(n);
  if (n) std::memcpy(v.data(), p, sizeof(T) * n);
  p += sizeof(T) * n;
  return v;
}
}  // namespace

void Metadata::Serialize(std::vector<char>* out) const {
  out->insert(out->end(), reinterpret_cast<const char*>(&num_data_), reinterpret_cast<const char*>(&num_data_) + 4);
  PutVec(out, label_);
  PutVec(out, weights_);
  PutVec(out, init_score_);
  PutVec(out, query_boundaries_);
  PutVec(out, positions_);
  int64_t np = static_cast<int64_t>(position_ids_.size());
  out->insert(out->end(), reinterpret_cast<const char*>(&np), reinterpret_cast<const char*>(&np) + 8);
  for (auto& s : position_ids_) {
    int64_t n = static_cast<int64_t>(s.size());
    out->insert(out->end(), reinterpret_cast<const char*>(&n), reinterpret_cast<const char*>(&n) + 8);
    out->insert(out->end(), s.begin(), s.end());
  }
}

size_t Metadata::Deserialize(const char* buf) {
  const char* p = buf;
  std::memcpy(&num_data_, p, 4);
  p += 4;
  label_ = GetVec<label_t>(p);
  weights_ = GetVec<label_t>(p);
  init_score_ = GetVec<double>(p);
  query_boundaries_ = GetVec<data_size_t>(p);
  positions_ = GetVec<int32_t>(p);
  int64_t np;
  std::memcpy(&np, p, 8);
  p += 8;
  position_ids_.clear();
  for (int64_t i = 0; i < np; ++i) {
    int64_t n;
    std::memcpy(&n, p, 8);
    p += 8;
    position_ids_.emplace_back(p, p + n);
    p += n;
  }
  CalcQueryWeights();
  return static_cast<size_t>(p - buf);
}

}  // namespace lgap
