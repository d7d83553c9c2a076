// Dataset construction: sampled bin finding, exclusive feature bundling,
// packed row-major bin matrix, subsets and the binary cache.
// Reference behaviour: src/io/dataset.cpp (FindGroups :107-244,
// FastFeatureBundling :246-323, Construct :325-441, SaveBinary :1018-1187) and
// dataset_loader.cpp:593 (ConstructFromSampleData).
#include "lgap/device_api.h"
#include "lgap/omp_errors.h"
#include "lgap/dataset.h"

#include <omp.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <numeric>
#include <set>

#include "lgap/common.h"
#include "lgap/log.h"
#include "lgap/network.h"
#include "lgap/random.h"

namespace lgap {

namespace {
const char* kBinaryToken = "______LambdaGap_Binary_File_Token______\n";
// zero rate from which a feature group is stored as multi-value sparse rows: an entry
// is 4 bytes against 1-2 per row densely, so this sits above the reference's
// kSparseThreshold (bin.h:43, 0.7)
constexpr double kSparseZeroRate = 0.8;

template <typename T>
void Put(std::vector<char>* out, const T& v) {
  const char* p = reinterpret_cast<const char*>(&v);
  out->insert(out->end(), p, p + sizeof(T));
}
template <typename T>
void PutVec(std::vector<char>* out, const std::vector<T>& v) {
  Put(out, static_cast<int64_t>(v.size()));
  const char* p = reinterpret_cast<const char*>(v.data());
  out->insert(out->end(), p, p + sizeof(T) * v.size());
}
template <typename T>
T Get(const char*& p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  p += sizeof(T);
  return v;
}
template <typename T>
std::vector<T> GetVec(const char*& p) {
  int64_t n = Get<int64_t>(p);
  std::vector<T> v(n);
  if (n) std::memcpy(v.data(), p, sizeof(T) * n);
  p += sizeof(T) * n;
  return v;
}
void PutStr(std::vector<char>* out, const std::string& s) {
  Put(out, static_cast<int64_t>(s.size()));
  out->insert(out->end(), s.begin(), s.end());
}
std::string GetStr(const char*& p) {
  int64_t n = Get<int64_t>(p);
  std::string s(p, p + n);
  p += n;
  return s;
}

std::vector<std::vector<double>> LoadForcedBins(const std::string& filename, int num_features) {
  std::vector<std::vector<double>> out(num_features);
  if (filename.empty()) return out;
  std::ifstream in(filename);
  if (!in) {
    Log::Warning("Forced bins file %s cannot be opened", filename.c_str());
    return out;
  }
  std::string text((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  // format: [{"feature": i, "bin_upper_bound": [..]}, ...]
  size_t pos = 0;
  while ((pos = text.find("\"feature\"", pos)) != std::string::npos) {
    size_t colon = text.find(':', pos);
    int f = static_cast<int>(std::strtol(text.c_str() + colon + 1, nullptr, 10));
    size_t ub = text.find("\"bin_upper_bound\"", colon);
    size_t lb = text.find('[', ub);
    size_t rb = text.find(']', lb);
    auto vals = common::StringToArray<double>(common::Trim(
        [&] { std::string s = text.substr(lb + 1, rb - lb - 1); for (auto& c : s) if (c == ',') c = ' '; return s; }()));
    if (f >= 0 && f < num_features) {
      std::sort(vals.begin(), vals.end());
      out[f] = vals;
    }
    pos = rb;
  }
  return out;
}
}  // namespace

// ---------------------------------------------------------------------------
void Dataset::set_feature_names(const std::vector<std::string>& n) {
  if (n.empty()) return;
  if (static_cast<int>(n.size()) != num_total_features_) {
    Log::Fatal("Length of feature_name(%d) and num_feature(%d) don't match", static_cast<int>(n.size()),
               num_total_features_);
  }
  feature_names_ = n;
  for (auto& s : feature_names_) {
    for (auto& c : s) if (c == ' ') c = '_';
  }
}

std::vector<std::string> Dataset::feature_infos() const {
  std::vector<std::string> out(num_total_features_);
  for (int i = 0; i < num_total_features_; ++i) {
    out[i] = used_map_[i] < 0 ? "none" : mappers_[i].bin_info_string();
  }
  return out;
}

std::string Dataset::reference_key() const {
  std::string k = std::to_string(num_total_features_) + ":" + std::to_string(num_total_bin_);
  return k;
}

bool Dataset::CheckAlign(const Dataset& o) const {
  if (num_total_features_ != o.num_total_features_ || features_.size() != o.features_.size()) return false;
  for (int i = 0; i < num_total_features_; ++i) {
    if (used_map_[i] != o.used_map_[i]) return false;
    if (used_map_[i] >= 0 && !mappers_[i].CheckAlign(o.mappers_[i])) return false;
  }
  return true;
}

void Dataset::BuildGroups(const Config& cfg, const std::vector<std::vector<int>>& nz_rows, data_size_t sample_cnt) {
  const int nf = num_features();
  groups_.clear();
  std::vector<std::vector<int>> best;
  auto find_groups = [&](const std::vector<int>& order) {
    const int max_bin_per_group = 256;
    const data_size_t max_conflict = sample_cnt / 10000;
    std::vector<std::vector<int>> grp;
    std::vector<std::vector<char>> marks;
    std::vector<data_size_t> used_rows, total_rows;
    std::vector<int> nbin;
    for (int f : order) {
      const int fb = features_[f].num_bin - 1;  // bins this feature adds
      const data_size_t nnz = static_cast<data_size_t>(nz_rows[f].size());
      int chosen = -1;
      int chosen_conf = 0;
      if (cfg.enable_bundle) {
        // search the most recent groups first (bounded search like the reference)
        int searched = 0;
        for (int g = static_cast<int>(grp.size()) - 1; g >= 0 && searched < 100; --g, ++searched) {
          if (nbin[g] + fb > max_bin_per_group) continue;
          if (total_rows[g] + nnz > sample_cnt + max_conflict) continue;
          data_size_t rest = max_conflict - total_rows[g] + used_rows[g];
          data_size_t conf = 0;
          bool ok = true;
          for (int r : nz_rows[f]) {
            if (marks[g][r]) {
              if (++conf > rest) { ok = false; break; }
            }
          }
          if (ok && conf <= nnz / 2) {
            chosen = g;
            chosen_conf = conf;
            break;
          }
        }
      }
      if (chosen >= 0) {
        grp[chosen].push_back(f);
        total_rows[chosen] += nnz;
        used_rows[chosen] += nnz - chosen_conf;
        for (int r : nz_rows[f]) marks[chosen][r] = 1;
        nbin[chosen] += fb;
      } else {
        grp.emplace_back(1, f);
        marks.emplace_back(sample_cnt, 0);
        for (int r : nz_rows[f]) marks.back()[r] = 1;
        total_rows.push_back(nnz);
        used_rows.push_back(nnz);
        nbin.push_back(1 + fb);
      }
    }
    return grp;
  };
  std::vector<int> order(nf);
  std::iota(order.begin(), order.end(), 0);
  if (!cfg.enable_bundle || nf <= 1) {
    for (int f : order) best.emplace_back(1, f);
  } else {
    best = find_groups(order);
    std::vector<int> by_cnt = order;
    std::stable_sort(by_cnt.begin(), by_cnt.end(),
                     [&](int a, int b) { return nz_rows[a].size() > nz_rows[b].size(); });
    auto g2 = find_groups(by_cnt);
    if (g2.size() < best.size()) best = g2;
    // keep a deterministic group order: by the smallest feature index in the group
    std::sort(best.begin(), best.end(), [](const std::vector<int>& a, const std::vector<int>& b) {
      return *std::min_element(a.begin(), a.end()) < *std::min_element(b.begin(), b.end());
    });
  }
  for (auto& g : best) {
    FeatureGroup fg;
    fg.features = g;
    groups_.push_back(fg);
  }
  if (groups_.size() < static_cast<size_t>(nf)) {
    Log::Info("EFB: bundled %d features into %d groups", nf, static_cast<int>(groups_.size()));
  }
}

void Dataset::FinalizeLayout() {
  num_total_bin_ = 0;
  bin_width_ = 1;
  for (int g = 0; g < num_groups(); ++g) {
    auto& fg = groups_[g];
    fg.hist_start = num_total_bin_;
    int off = 1;
    for (int f : fg.features) {
      auto& fi = features_[f];
      fi.group = g;
      fi.offset = off;
      fi.hist_offset = fg.hist_start + off;
      off += fi.num_bin - 1;
    }
    fg.num_bin = off;
    if (fg.num_bin > 256) bin_width_ = 2;
    if (fg.num_bin > 65536) Log::Fatal("Feature group with %d bins exceeds 65536", fg.num_bin);
    num_total_bin_ += fg.num_bin;
  }
  // pad each row to a multiple of 4 bytes (dword-aligned records for the device kernels)
  row_stride_ = FullStride(num_groups(), bin_width_);
  num_dense_groups_ = num_groups();
  sp_ptr_.clear();
  sp_bin_.clear();
}

// Multi-value sparse storage (reference src/io/multi_val_sparse_bin.hpp and the
// is_multi_val feature groups of dataset.cpp:219-242 / feature_group.h:216). A group whose
// rows are at least `zero_threshold` at group bin 0 moves out of the dense matrix into one
// CSR of global histogram bins; the host row-wise histogram then walks only its non-zeros.
// Sparse groups are moved to the end of the group order (dense groups keep their order),
// so a dense row keeps the layout the device kernels expect for its leading groups and a
// full row (MaterializeRows) is the dense row followed by the sparse groups' bins.
// Per-bin sums are accumulated in the same row order either way: models are identical.
void Dataset::CompressSparseGroups(double zero_threshold) {
  const int ng = num_groups();
  if (ng == 0 || num_data_ <= 0 || has_sparse()) return;
  std::vector<data_size_t> nnz(ng, 0);
#pragma omp parallel
  {
    std::vector<data_size_t> local(ng, 0);
#pragma omp for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      for (int g = 0; g < ng; ++g) local[g] += GroupBin(i, g) != 0u;
    }
#pragma omp critical
    for (int g = 0; g < ng; ++g) nnz[g] += local[g];
  }
  std::vector<int> order, sparse;
  for (int g = 0; g < ng; ++g) {
    const double zero_rate = 1.0 - static_cast<double>(nnz[g]) / num_data_;
    (zero_rate >= zero_threshold ? sparse : order).push_back(g);
  }
  if (sparse.empty()) return;
  const int nd = static_cast<int>(order.size());
  order.insert(order.end(), sparse.begin(), sparse.end());
  const std::vector<uint8_t> old_bins = std::move(bins_);
  const int old_stride = row_stride_, width = bin_width_;
  std::vector<FeatureGroup> ng_groups;
  for (int g : order) ng_groups.push_back(groups_[g]);
  groups_.swap(ng_groups);
  FinalizeLayout();
  bin_width_ = width;
  num_dense_groups_ = nd;
  row_stride_ = FullStride(nd, width);
  auto old_bin = [&](data_size_t i, int g) -> uint32_t {
    const uint8_t* r = old_bins.data() + static_cast<size_t>(i) * old_stride;
    return width == 1 ? r[g] : reinterpret_cast<const uint16_t*>(r)[g];
  };
  bins_.assign(static_cast<size_t>(num_data_) * row_stride_, 0);
  sp_ptr_.assign(static_cast<size_t>(num_data_) + 1, 0);
#pragma omp parallel for schedule(static)
  for (data_size_t i = 0; i < num_data_; ++i) {
    uint8_t* r = bins_.data() + static_cast<size_t>(i) * row_stride_;
    for (int j = 0; j < nd; ++j) {
      const uint32_t v = old_bin(i, order[j]);
      if (width == 1) r[j] = static_cast<uint8_t>(v);
      else reinterpret_cast<uint16_t*>(r)[j] = static_cast<uint16_t>(v);
    }
    uint64_t c = 0;
    for (int j = nd; j < ng; ++j) c += old_bin(i, order[j]) != 0u;
    sp_ptr_[static_cast<size_t>(i) + 1] = c;
  }
  for (data_size_t i = 0; i < num_data_; ++i) sp_ptr_[static_cast<size_t>(i) + 1] += sp_ptr_[i];
  sp_bin_.resize(sp_ptr_.back());
#pragma omp parallel for schedule(static)
  for (data_size_t i = 0; i < num_data_; ++i) {
    uint64_t k = sp_ptr_[i];
    for (int j = nd; j < ng; ++j) {  // hist_start ascends with j: entries stay sorted
      const uint32_t v = old_bin(i, order[j]);
      if (v != 0u) sp_bin_[k++] = static_cast<uint32_t>(groups_[j].hist_start) + v;
    }
  }
  Log::Info("Sparse storage: %d of %d feature groups as multi-value sparse rows (%.2f non-zeros per row)",
            ng - nd, ng, static_cast<double>(sp_bin_.size()) / num_data_);
}

void Dataset::MaterializeRows(std::vector<uint8_t>* out) const {
  const int fs = row_stride(), ng = num_groups(), nd = num_dense_groups_;
  out->assign(static_cast<size_t>(num_data_) * fs, 0);
  std::vector<uint32_t> sstart;
  for (int g = nd; g < ng; ++g) sstart.push_back(static_cast<uint32_t>(groups_[g].hist_start));
  const int dense_bytes = nd * bin_width_;
#pragma omp parallel for schedule(static)
  for (data_size_t i = 0; i < num_data_; ++i) {
    uint8_t* r = out->data() + static_cast<size_t>(i) * fs;
    std::memcpy(r, bins_.data() + static_cast<size_t>(i) * row_stride_, dense_bytes);
    if (sp_ptr_.empty()) continue;
    for (uint64_t k = sp_ptr_[i]; k < sp_ptr_[static_cast<size_t>(i) + 1]; ++k) {
      const uint32_t e = sp_bin_[k];
      const int j = static_cast<int>(std::upper_bound(sstart.begin(), sstart.end(), e) - sstart.begin()) - 1;
      const int g = nd + j;
      const uint32_t v = e - sstart[j];
      if (bin_width_ == 1) r[g] = static_cast<uint8_t>(v);
      else reinterpret_cast<uint16_t*>(r)[g] = static_cast<uint16_t>(v);
    }
  }
}

const uint8_t* Dataset::RowsForDevice(std::vector<uint8_t>* scratch) const {
  if (!has_sparse()) return bins_.data();
  MaterializeRows(scratch);
  return scratch->data();
}

void Dataset::Densify() {
  if (!has_sparse()) return;
  std::vector<uint8_t> full;
  MaterializeRows(&full);
  bins_.swap(full);
  row_stride_ = FullStride(num_groups(), bin_width_);
  num_dense_groups_ = num_groups();
  sp_ptr_.clear();
  sp_bin_.clear();
}

void Dataset::InitEmptyLike(const Dataset& ref, data_size_t n) {
  num_data_ = n;
  num_total_features_ = ref.num_total_features_;
  feature_names_ = ref.feature_names_;
  mappers_ = ref.mappers_;
  used_map_ = ref.used_map_;
  features_ = ref.features_;
  groups_ = ref.groups_;
  categorical_ = ref.categorical_;
  num_total_bin_ = ref.num_total_bin_;
  bin_width_ = ref.bin_width_;
  row_stride_ = FullStride(num_groups(), bin_width_);  // streamed rows are stored dense
  num_dense_groups_ = num_groups();
  bins_.assign(static_cast<size_t>(n) * row_stride_, 0);
  metadata_.Init(n);
}

void Dataset::PushRows(const RowSource& src, data_size_t start_row) {
  if (start_row + src.num_rows() > num_data_) Log::Fatal("Pushed rows exceed the dataset size");
  PackRows(src, start_row, false);
}

Dataset::~Dataset() { device::ReleaseDeviceRows(this); }

void Dataset::PackRows(const RowSource& src, data_size_t start_row, bool reset) {
  const data_size_t nrows = src.num_rows();
  if (reset) {
    num_data_ = nrows;
    bins_.assign(static_cast<size_t>(num_data_) * row_stride_, 0);
    if (keep_raw_) raw_.assign(static_cast<size_t>(num_data_) * features_.size(), 0.0f);
  }
  // device binning of a dense row-major matrix (bin_kernels.hip); the device rows are kept
  // for the HIP learner. Anything else (sparse / Arrow / streaming / raw values) bins here.
  const auto* dense = dynamic_cast<const DenseSource*>(&src);
  if (device_pack_ && reset && start_row == 0 && !keep_raw_ && dense != nullptr && dense->row_major() &&
      device::DeviceCount() > 0 &&
      device::DevicePackDense(*this, dense->data(), dense->is_f64(), nrows, dense->num_cols(), bins_.data(), true)) {
    return;
  }
  const size_t nfeat = features_.size();
  const bool store_raw = keep_raw_ && !raw_.empty();
  // template row: bins when every value is zero
  std::vector<uint8_t> tmpl(row_stride_, 0);
  std::vector<int> owner(num_groups(), -1);
  for (int f = 0; f < num_features(); ++f) {
    const auto& fi = features_[f];
    if (fi.default_bin != fi.mfb) {
      int gb = EncodeBin(fi, fi.default_bin);
      if (bin_width_ == 1) tmpl[fi.group] = static_cast<uint8_t>(gb);
      else reinterpret_cast<uint16_t*>(tmpl.data())[fi.group] = static_cast<uint16_t>(gb);
      owner[fi.group] = f;
    }
  }
  const int nthreads = omp_get_max_threads();
  OmpErrors errs;  // row sources (Arrow, Python sequences through the C API) may raise
#pragma omp parallel num_threads(nthreads)
  {
    std::vector<std::pair<int, double>> row;
#pragma omp for schedule(static, 4096)
    for (data_size_t i = 0; i < nrows; ++i) {
      errs.Run([&] {
        uint8_t* r = bins_.data() + static_cast<size_t>(i + start_row) * row_stride_;
        std::memcpy(r, tmpl.data(), row_stride_);
        src.GetRow(i, &row);
        for (auto& kv : row) {
          if (kv.first >= num_total_features_) continue;
          int f = used_map_[kv.first];
          if (f < 0) continue;
          const auto& fi = features_[f];
          if (store_raw) raw_[static_cast<size_t>(i + start_row) * nfeat + f] = static_cast<float>(kv.second);
          uint32_t b = mappers_[kv.first].ValueToBin(kv.second);
          int gb = EncodeBin(fi, b);
          if (gb == 0 && owner[fi.group] != f) continue;
          if (bin_width_ == 1) r[fi.group] = static_cast<uint8_t>(gb);
          else reinterpret_cast<uint16_t*>(r)[fi.group] = static_cast<uint16_t>(gb);
        }
      });
    }
  }
  errs.Rethrow();
}

void Dataset::Construct(const RowSource& src, const Config& cfg, const Dataset* reference,
                        const std::vector<std::string>& names, const std::vector<int>& categorical) {
  ScopedTimer t("Dataset::Construct");
  num_data_ = src.num_rows();
  num_total_features_ = src.num_cols();
  keep_raw_ = cfg.linear_tree || (reference != nullptr && reference->keep_raw_);
  // device binning keeps its packed rows for the learner to adopt: training sets only (a
  // validation set's rows are uploaded by DeviceAddValidSet, a kept copy would sit unused)
  device_pack_ = (cfg.device_type == "gpu" || cfg.device_type == "cuda") && cfg.device_binning && reference == nullptr;
  if (reference != nullptr) {
    if (reference->num_total_features_ != num_total_features_) {
      Log::Fatal("The number of features in data (%d) is not the same as it was in training data (%d).",
                 num_total_features_, reference->num_total_features_);
    }
    mappers_ = reference->mappers_;
    used_map_ = reference->used_map_;
    features_ = reference->features_;
    groups_ = reference->groups_;
    categorical_ = reference->categorical_;
    feature_names_ = reference->feature_names_;
    num_total_bin_ = reference->num_total_bin_;
    bin_width_ = reference->bin_width_;
    row_stride_ = FullStride(num_groups(), bin_width_);  // the reference's groups, stored dense
    num_dense_groups_ = num_groups();
    PackRows(src);
    metadata_.Init(num_data_);
    return;
  }
  feature_names_.resize(num_total_features_);
  for (int i = 0; i < num_total_features_; ++i) feature_names_[i] = "Column_" + std::to_string(i);
  if (!names.empty()) set_feature_names(names);
  categorical_ = categorical;
  std::set<int> cat_set(categorical.begin(), categorical.end());

  // ---- sample rows for bin construction
  const data_size_t sample_cnt = std::min<data_size_t>(num_data_, cfg.bin_construct_sample_cnt);
  Random rand(cfg.data_random_seed);
  std::vector<int> sample_idx = rand.Sample(num_data_, sample_cnt);
  std::vector<std::vector<double>> col_vals(num_total_features_);
  std::vector<std::vector<int>> col_rows(num_total_features_);
  {
    std::vector<std::pair<int, double>> row;
    for (int s = 0; s < static_cast<int>(sample_idx.size()); ++s) {
      src.GetRow(sample_idx[s], &row);
      for (auto& kv : row) {
        if (kv.first >= num_total_features_) continue;
        col_vals[kv.first].push_back(kv.second);
        col_rows[kv.first].push_back(s);
      }
    }
  }
  auto forced = LoadForcedBins(cfg.forcedbins_filename, num_total_features_);
  mappers_.assign(num_total_features_, BinMapper());
  std::vector<char> ignore(num_total_features_, 0);
  if (!cfg.ignore_column.empty()) {
    // numeric indices only at this level (names are resolved by the loader)
    for (auto& tok : common::Split(cfg.ignore_column, ',')) {
      if (!tok.empty() && std::isdigit(static_cast<unsigned char>(tok[0]))) {
        int c = common::AtoiOrDie(tok);
        if (c >= 0 && c < num_total_features_) ignore[c] = 1;
      }
    }
  }
  OmpErrors errs;  // FindBin rejects invalid bin settings with Log::Fatal
#pragma omp parallel for schedule(dynamic)
  for (int j = 0; j < num_total_features_; ++j) {
    if (ignore[j] || errs.failed()) continue;
    try {
    int mb = cfg.max_bin;
    if (!cfg.max_bin_by_feature.empty()) {
      if (static_cast<int>(cfg.max_bin_by_feature.size()) != num_total_features_) {
        mb = cfg.max_bin;
      } else {
        mb = cfg.max_bin_by_feature[j];
      }
    }
    std::vector<double> vals = col_vals[j];
    mappers_[j].FindBin(vals.data(), static_cast<int>(vals.size()), sample_idx.size(), mb, cfg.min_data_in_bin,
                        cfg.min_data_in_leaf, cfg.feature_pre_filter,
                        cat_set.count(j) ? BinType::Categorical : BinType::Numerical, cfg.use_missing,
                        cfg.zero_as_missing, forced[j]);
    } catch (...) {
      errs.Capture();
    }
  }
  errs.Rethrow();
  // ---- distributed: every rank adopts the mappers of the feature's owner rank
  // (features dealt round-robin; reference dataset_loader.cpp:1166-1262 splits
  // the feature range and allgathers serialized BinMappers the same way).
  const int nm = Network::num_machines();
  if (nm > 1) {
    std::vector<char> mine;
    for (int j = Network::rank(); j < num_total_features_; j += nm) mappers_[j].Serialize(&mine);
    auto blobs = Network::AllgatherBlobs(mine);
    for (int r = 0; r < nm; ++r) {
      const char* p = blobs[r].data();
      for (int j = r; j < num_total_features_; j += nm) p += mappers_[j].Deserialize(p);
    }
  }
  // ---- used features
  used_map_.assign(num_total_features_, -1);
  features_.clear();
  for (int j = 0; j < num_total_features_; ++j) {
    if (ignore[j] || mappers_[j].is_trivial()) continue;
    FeatureInfo fi;
    fi.real_index = j;
    fi.num_bin = mappers_[j].num_bin();
    fi.mfb = mappers_[j].most_freq_bin();
    fi.default_bin = mappers_[j].default_bin();
    fi.missing = mappers_[j].missing_type();
    fi.bin_type = mappers_[j].bin_type();
    if (!cfg.monotone_constraints.empty() && j < static_cast<int>(cfg.monotone_constraints.size())) {
      fi.monotone = cfg.monotone_constraints[j];
    }
    if (!cfg.feature_contri.empty() && j < static_cast<int>(cfg.feature_contri.size())) {
      fi.penalty = cfg.feature_contri[j];
    }
    used_map_[j] = static_cast<int>(features_.size());
    features_.push_back(fi);
  }
  if (features_.empty()) {
    Log::Warning("There are no meaningful features which satisfy the provided configuration. "
                 "Decreasing Dataset parameters min_data_in_bin or min_data_in_leaf and re-constructing "
                 "Dataset might resolve this warning.");
  }
  // ---- non-mfb sample rows per used feature (for EFB conflict counting)
  std::vector<std::vector<int>> nz(features_.size());
#pragma omp parallel for schedule(dynamic)
  for (int f = 0; f < static_cast<int>(features_.size()); ++f) {
    const int j = features_[f].real_index;
    const auto& m = mappers_[j];
    if (m.default_bin() == m.most_freq_bin()) {
      for (size_t k = 0; k < col_rows[j].size(); ++k) {
        if (m.ValueToBin(col_vals[j][k]) != m.most_freq_bin()) nz[f].push_back(col_rows[j][k]);
      }
    } else {
      // zeros are non-mfb too: all sampled rows except those whose value maps to mfb
      size_t k = 0;
      for (int s = 0; s < static_cast<int>(sample_idx.size()); ++s) {
        if (k < col_rows[j].size() && col_rows[j][k] == s) {
          if (m.ValueToBin(col_vals[j][k]) != m.most_freq_bin()) nz[f].push_back(s);
          ++k;
        } else {
          nz[f].push_back(s);
        }
      }
    }
  }
  BuildGroups(cfg, nz, static_cast<data_size_t>(sample_idx.size()));
  if (nm > 1) {
    // bundles were decided on local samples: adopt rank 0's so histogram layouts agree
    std::vector<char> mine;
    if (Network::rank() == 0) {
      auto put = [&mine](int v) { mine.insert(mine.end(), reinterpret_cast<char*>(&v), reinterpret_cast<char*>(&v) + 4); };
      put(static_cast<int>(groups_.size()));
      for (auto& g : groups_) {
        put(static_cast<int>(g.features.size()));
        for (int f : g.features) put(f);
      }
    }
    auto blobs = Network::AllgatherBlobs(mine);
    const char* p = blobs[0].data();
    auto get = [&p]() {
      int v;
      std::memcpy(&v, p, 4);
      p += 4;
      return v;
    };
    groups_.assign(get(), FeatureGroup());
    for (auto& g : groups_) {
      g.features.resize(get());
      for (auto& f : g.features) f = get();
    }
  }
  FinalizeLayout();
  PackRows(src);
  metadata_.Init(num_data_);
  // single-process host training only: ranks would choose different sparse sets (their own
  // rows) and the device kernels stream dense rows
  if (cfg.is_enable_sparse && !device_pack_ && nm == 1 && cfg.device_type == "cpu" && cfg.num_machines <= 1) {
    CompressSparseGroups(kSparseZeroRate);
  }
}

void Dataset::ConstructFromMappers(std::vector<BinMapper> mappers, const RowSource& src, const Config& cfg,
                                   const std::vector<std::string>& names) {
  num_data_ = src.num_rows();
  num_total_features_ = static_cast<int>(mappers.size());
  mappers_ = std::move(mappers);
  feature_names_.resize(num_total_features_);
  for (int i = 0; i < num_total_features_; ++i) feature_names_[i] = "Column_" + std::to_string(i);
  if (!names.empty()) set_feature_names(names);
  used_map_.assign(num_total_features_, -1);
  features_.clear();
  for (int j = 0; j < num_total_features_; ++j) {
    if (mappers_[j].is_trivial()) continue;
    FeatureInfo fi;
    fi.real_index = j;
    fi.num_bin = mappers_[j].num_bin();
    fi.mfb = mappers_[j].most_freq_bin();
    fi.default_bin = mappers_[j].default_bin();
    fi.missing = mappers_[j].missing_type();
    fi.bin_type = mappers_[j].bin_type();
    if (fi.bin_type == BinType::Categorical) categorical_.push_back(j);
    if (!cfg.monotone_constraints.empty() && j < static_cast<int>(cfg.monotone_constraints.size()))
      fi.monotone = cfg.monotone_constraints[j];
    if (!cfg.feature_contri.empty() && j < static_cast<int>(cfg.feature_contri.size()))
      fi.penalty = cfg.feature_contri[j];
    used_map_[j] = static_cast<int>(features_.size());
    features_.push_back(fi);
  }
  groups_.clear();
  for (int f = 0; f < num_features(); ++f) {
    FeatureGroup g;
    g.features = {f};
    groups_.push_back(g);
  }
  FinalizeLayout();
  PackRows(src);
  metadata_.Init(num_data_);
}

void Dataset::FeatureHistogram(const double* gh, int f, double sum_g, double sum_h, double* out) const {
  const FeatureInfo& fi = features_[f];
  double sg = 0.0, sh = 0.0;
  for (int b = 0, k = 0; b < fi.num_bin; ++b) {
    if (static_cast<uint32_t>(b) == fi.mfb) continue;
    double g = gh[2 * (fi.hist_offset + k)];
    double h = gh[2 * (fi.hist_offset + k) + 1];
    out[2 * b] = g;
    out[2 * b + 1] = h;
    sg += g;
    sh += h;
    ++k;
  }
  out[2 * fi.mfb] = sum_g - sg;
  out[2 * fi.mfb + 1] = sum_h - sh;
}

std::unique_ptr<Dataset> Dataset::Subset(const std::vector<data_size_t>& idx) const {
  auto d = std::make_unique<Dataset>();
  d->num_data_ = static_cast<data_size_t>(idx.size());
  d->num_total_features_ = num_total_features_;
  d->feature_names_ = feature_names_;
  d->mappers_ = mappers_;
  d->used_map_ = used_map_;
  d->features_ = features_;
  d->groups_ = groups_;
  d->categorical_ = categorical_;
  d->num_total_bin_ = num_total_bin_;
  d->bin_width_ = bin_width_;
  d->row_stride_ = row_stride_;
  d->num_dense_groups_ = num_dense_groups_;
  d->bins_.resize(static_cast<size_t>(d->num_data_) * row_stride_);
#pragma omp parallel for schedule(static)
  for (data_size_t i = 0; i < d->num_data_; ++i) {
    std::memcpy(d->bins_.data() + static_cast<size_t>(i) * row_stride_,
                bins_.data() + static_cast<size_t>(idx[i]) * row_stride_, row_stride_);
  }
  if (!sp_ptr_.empty()) {
    d->sp_ptr_.assign(static_cast<size_t>(d->num_data_) + 1, 0);
    for (data_size_t i = 0; i < d->num_data_; ++i) {
      d->sp_ptr_[static_cast<size_t>(i) + 1] = d->sp_ptr_[i] + sp_ptr_[static_cast<size_t>(idx[i]) + 1] - sp_ptr_[idx[i]];
    }
    d->sp_bin_.resize(d->sp_ptr_.back());
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < d->num_data_; ++i) {
      std::copy(sp_bin_.begin() + sp_ptr_[idx[i]], sp_bin_.begin() + sp_ptr_[static_cast<size_t>(idx[i]) + 1],
                d->sp_bin_.begin() + d->sp_ptr_[i]);
    }
  }
  d->metadata_.Subset(metadata_, idx.data(), d->num_data_);
  return d;
}

void Dataset::AddFeaturesFrom(const Dataset& o) {
  if (o.num_data_ != num_data_) Log::Fatal("Cannot add features from other Dataset with a different number of rows");
  Densify();
  const int old_groups = num_groups();
  const int old_stride = row_stride_;
  const int old_width = bin_width_;
  std::set<std::string> taken(feature_names_.begin(), feature_names_.end());
  for (int j = 0; j < o.num_total_features_; ++j) {
    mappers_.push_back(o.mappers_[j]);
    // a clashing name becomes D<k>_<name> with the first free k >= 2 (as the reference)
    std::string name = o.feature_names_[j];
    for (int k = 2; taken.count(name); ++k) name = "D" + std::to_string(k) + "_" + o.feature_names_[j];
    if (name != o.feature_names_[j]) {
      Log::Warning("Find the same feature name (%s) in Dataset::AddFeaturesFrom, change its name to (%s)",
                   o.feature_names_[j].c_str(), name.c_str());
    }
    taken.insert(name);
    feature_names_.push_back(name);
    used_map_.push_back(o.used_map_[j] < 0 ? -1 : o.used_map_[j] + static_cast<int>(features_.size()));
  }
  const int fbase = static_cast<int>(features_.size());
  for (auto fi : o.features_) {
    fi.real_index += num_total_features_;
    features_.push_back(fi);
  }
  for (auto g : o.groups_) {
    for (auto& f : g.features) f += fbase;
    groups_.push_back(g);
  }
  for (int c : o.categorical_) categorical_.push_back(c + num_total_features_);
  num_total_features_ += o.num_total_features_;
  FinalizeLayout();
  std::vector<uint8_t> nb(static_cast<size_t>(num_data_) * row_stride_, 0);
  for (data_size_t i = 0; i < num_data_; ++i) {
    uint8_t* r = nb.data() + static_cast<size_t>(i) * row_stride_;
    for (int g = 0; g < num_groups(); ++g) {
      uint32_t v;
      if (g < old_groups) {
        const uint8_t* src = bins_.data() + static_cast<size_t>(i) * old_stride;
        v = old_width == 1 ? src[g] : reinterpret_cast<const uint16_t*>(src)[g];
      } else {
        v = o.GroupBin(i, g - old_groups);
      }
      if (bin_width_ == 1) r[g] = static_cast<uint8_t>(v);
      else reinterpret_cast<uint16_t*>(r)[g] = static_cast<uint16_t>(v);
    }
  }
  bins_.swap(nb);
}

// ---------------------------------------------------------------------------
bool Dataset::IsBinaryFile(const std::string& filename) {
  std::ifstream in(filename, std::ios::binary);
  if (!in) return false;
  std::string tok(std::strlen(kBinaryToken), '\0');
  in.read(&tok[0], tok.size());
  return in.gcount() == static_cast<std::streamsize>(tok.size()) && tok == kBinaryToken;
}

void Dataset::SerializeBinary(std::vector<char>* out) const {
  std::vector<char>& buf = *out;
  buf.assign(kBinaryToken, kBinaryToken + std::strlen(kBinaryToken));
  Put(&buf, num_data_);
  Put(&buf, num_total_features_);
  Put(&buf, num_total_bin_);
  Put(&buf, bin_width_);
  Put(&buf, row_stride_);
  Put(&buf, static_cast<int32_t>(feature_names_.size()));
  for (auto& n : feature_names_) PutStr(&buf, n);
  for (auto& m : mappers_) m.Serialize(&buf);
  PutVec(&buf, used_map_);
  Put(&buf, static_cast<int32_t>(features_.size()));
  for (auto& f : features_) Put(&buf, f);
  Put(&buf, static_cast<int32_t>(groups_.size()));
  for (auto& g : groups_) {
    Put(&buf, g.num_bin);
    Put(&buf, g.hist_start);
    PutVec(&buf, g.features);
  }
  PutVec(&buf, categorical_);
  metadata_.Serialize(&buf);
  PutVec(&buf, bins_);
  // raw feature values (linear_tree): the reference's binary format stores them too
  // (dataset.cpp SaveBinaryFile, raw_data_ section)
  Put(&buf, static_cast<int32_t>(keep_raw_ ? 1 : 0));
  PutVec(&buf, raw_);
  // multi-value sparse groups (absent in files written before the sparse storage)
  Put(&buf, static_cast<int32_t>(num_dense_groups_));
  PutVec(&buf, sp_ptr_);
  PutVec(&buf, sp_bin_);
}

void Dataset::SaveBinary(const std::string& filename) const {
  std::vector<char> buf;
  SerializeBinary(&buf);
  std::ofstream out(filename, std::ios::binary);
  if (!out) Log::Fatal("Cannot write binary data to %s", filename.c_str());
  out.write(buf.data(), buf.size());
  Log::Info("Saving data to binary file %s", filename.c_str());
}

std::unique_ptr<Dataset> Dataset::LoadBinary(const std::string& filename) {
  std::ifstream in(filename, std::ios::binary);
  if (!in) Log::Fatal("Cannot open binary file %s", filename.c_str());
  std::vector<char> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (buf.size() < std::strlen(kBinaryToken) || std::memcmp(buf.data(), kBinaryToken, std::strlen(kBinaryToken)) != 0) {
    Log::Fatal("File %s is not a LambdaGap binary dataset", filename.c_str());
  }
  return DeserializeBinary(buf.data(), buf.size());
}

std::unique_ptr<Dataset> Dataset::DeserializeBinary(const char* data, size_t size) {
  const char* p = data;
  if (size < std::strlen(kBinaryToken) || std::memcmp(p, kBinaryToken, std::strlen(kBinaryToken)) != 0) {
    Log::Fatal("Buffer is not a serialized LambdaGap dataset");
  }
  p += std::strlen(kBinaryToken);
  auto d = std::make_unique<Dataset>();
  d->num_data_ = Get<data_size_t>(p);
  d->num_total_features_ = Get<int>(p);
  d->num_total_bin_ = Get<int>(p);
  d->bin_width_ = Get<int>(p);
  d->row_stride_ = Get<int>(p);
  int nn = Get<int32_t>(p);
  for (int i = 0; i < nn; ++i) d->feature_names_.push_back(GetStr(p));
  d->mappers_.resize(d->num_total_features_);
  for (auto& m : d->mappers_) p += m.Deserialize(p);
  d->used_map_ = GetVec<int>(p);
  int nf = Get<int32_t>(p);
  d->features_.resize(nf);
  for (auto& f : d->features_) f = Get<FeatureInfo>(p);
  int ng = Get<int32_t>(p);
  d->groups_.resize(ng);
  for (auto& g : d->groups_) {
    g.num_bin = Get<int>(p);
    g.hist_start = Get<int>(p);
    g.features = GetVec<int>(p);
  }
  d->categorical_ = GetVec<int>(p);
  p += d->metadata_.Deserialize(p);
  d->bins_ = GetVec<uint8_t>(p);
  d->num_dense_groups_ = ng;
  if (p < data + size) {
    d->keep_raw_ = Get<int32_t>(p) != 0;
    d->raw_ = GetVec<float>(p);
  }
  if (p < data + size) {
    d->num_dense_groups_ = Get<int32_t>(p);
    d->sp_ptr_ = GetVec<uint64_t>(p);
    d->sp_bin_ = GetVec<uint32_t>(p);
  }
  return d;
}

}  // namespace lgap
