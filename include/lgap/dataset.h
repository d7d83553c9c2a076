// Binned training data. Layout is MI355X-first: one packed row-major matrix
// of "group bins" (uint8, or uint16 when any group needs >256 bins), so a row
// is a contiguous record that the HIP histogram kernel streams with 16-byte
// loads and the partition kernel moves as a unit.
//
// Every feature's most-frequent bin (mfb) is *implicit*: a group bin of 0
// means "all features of this group at their mfb", and feature f occupies
// group bins [offset_f, offset_f + num_bin_f - 1). Histograms therefore never
// accumulate the most-frequent bin (the most contended LDS address) and it is
// reconstructed as leaf_total - sum(other bins) — the reference's FixHistogram
// / offset trick (dataset.cpp:1488-1506, feature_histogram.hpp:1429-1433)
// applied uniformly. EFB bundles (dataset.cpp:107-323) share one group.
#pragma once

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "lgap/bin.h"
#include "lgap/config.h"
#include "lgap/meta.h"

namespace lgap {

class Metadata {
 public:
  void Init(data_size_t num_data, int num_class_init_score = 0);
  void SetLabel(const float* label, data_size_t len);
  void SetWeights(const float* w, data_size_t len);
  void SetInitScore(const double* s, size_t len);
  void SetQuery(const data_size_t* group_sizes, data_size_t num_groups);  // sizes per query
  void SetQueryBoundaries(const std::vector<data_size_t>& b);
  void SetPosition(const int32_t* pos, data_size_t len);
  void Subset(const Metadata& src, const data_size_t* idx, data_size_t n);
  // streaming pushes: rows [start, start + n) (query = per-row query ids; boundaries are
  // derived once the last row has arrived)
  void SetRows(data_size_t start, data_size_t n, const float* label, const float* weight, const double* init_score,
               const int32_t* query);

  data_size_t num_data() const { return num_data_; }
  const label_t* label() const { return label_.data(); }
  const std::vector<label_t>& label_vec() const { return label_; }
  const label_t* weights() const { return weights_.empty() ? nullptr : weights_.data(); }
  const std::vector<label_t>& weights_vec() const { return weights_; }
  const double* init_score() const { return init_score_.empty() ? nullptr : init_score_.data(); }
  size_t init_score_size() const { return init_score_.size(); }
  const data_size_t* query_boundaries() const { return query_boundaries_.empty() ? nullptr : query_boundaries_.data(); }
  data_size_t num_queries() const { return query_boundaries_.empty() ? 0 : static_cast<data_size_t>(query_boundaries_.size()) - 1; }
  const label_t* query_weights() const { return query_weights_.empty() ? nullptr : query_weights_.data(); }
  const int32_t* positions() const { return positions_.empty() ? nullptr : positions_.data(); }
  const std::vector<std::string>& position_ids() const { return position_ids_; }
  int num_position_ids() const { return static_cast<int>(position_ids_.size()); }
  const std::vector<data_size_t>& query_boundaries_vec() const { return query_boundaries_; }

  void LoadSideFiles(const std::string& data_filename);  // .weight .query .init .position
  void Serialize(std::vector<char>* out) const;
  size_t Deserialize(const char* p);
  void CheckOrPartition(data_size_t num_all, const std::vector<data_size_t>& used_indices);

 private:
  void CalcQueryWeights();
  std::vector<int32_t> pending_query_ids_;
  data_size_t num_data_ = 0;
  std::vector<label_t> label_;
  std::vector<label_t> weights_;
  std::vector<double> init_score_;
  std::vector<data_size_t> query_boundaries_;
  std::vector<label_t> query_weights_;
  std::vector<int32_t> positions_;
  std::vector<std::string> position_ids_;
};

// Per used ("inner") feature description.
struct FeatureInfo {
  int real_index = 0;        // column in the user's matrix
  int group = 0;
  int offset = 1;            // first group bin of this feature
  int num_bin = 0;
  uint32_t mfb = 0;          // most frequent bin, implicit in histograms
  uint32_t default_bin = 0;  // bin of value 0
  MissingType missing = MissingType::None;
  BinType bin_type = BinType::Numerical;
  int8_t monotone = 0;
  double penalty = 1.0;
  int hist_offset = 0;       // global histogram position of group bin `offset`
};

struct FeatureGroup {
  int num_bin = 1;                // total group bins, incl. the shared zero bin
  int hist_start = 0;             // start of this group in the global histogram
  std::vector<int> features;      // inner feature indices
};

// Column-source abstraction used to build a Dataset from dense / CSR / CSC input.
struct RowSource {
  virtual ~RowSource() = default;
  virtual data_size_t num_rows() const = 0;
  virtual int num_cols() const = 0;
  // Writes the non-zero (or NaN) entries of row i as (col, value) pairs.
  virtual void GetRow(data_size_t i, std::vector<std::pair<int, double>>* out) const = 0;
};

class Dataset {
 public:
  Dataset() = default;
  ~Dataset();
  Dataset(const Dataset&) = default;
  Dataset& operator=(const Dataset&) = default;
  Dataset(Dataset&&) = default;
  Dataset& operator=(Dataset&&) = default;

  // Build bin mappers from a sample + pack all rows (c_api.cpp:1322 / dataset_loader.cpp:593 analogue).
  void Construct(const RowSource& src, const Config& cfg, const Dataset* reference,
                 const std::vector<std::string>& feature_names, const std::vector<int>& categorical);
  // Build from pre-computed bin mappers (distributed bin finding, binary cache).
  void ConstructFromMappers(std::vector<BinMapper> mappers, const RowSource& src, const Config& cfg,
                            const std::vector<std::string>& feature_names);
  std::unique_ptr<Dataset> Subset(const std::vector<data_size_t>& idx) const;

  void SaveBinary(const std::string& filename) const;
  static std::unique_ptr<Dataset> LoadBinary(const std::string& filename);
  // custom parser config (parser_config_file) the rows were parsed with; kept in the model
  const std::string& parser_config() const { return parser_config_; }
  void set_parser_config(const std::string& c) { parser_config_ = c; }
  // in-memory form of the binary file (LGBM_DatasetSerializeReferenceToBinary)
  void SerializeBinary(std::vector<char>* out) const;
  static std::unique_ptr<Dataset> DeserializeBinary(const char* data, size_t size);
  static bool IsBinaryFile(const std::string& filename);

  data_size_t num_data() const { return num_data_; }
  int num_total_features() const { return num_total_features_; }
  int num_features() const { return static_cast<int>(features_.size()); }
  int num_groups() const { return static_cast<int>(groups_.size()); }
  int num_total_bin() const { return num_total_bin_; }
  int bin_width() const { return bin_width_; }
  // stride of a row with EVERY group packed (the device kernels' record; MaterializeRows)
  int row_stride() const { return FullStride(num_groups(), bin_width_); }
  // the stored dense part: groups [0, num_dense_groups()) packed row-major at dense_stride()
  int num_dense_groups() const { return num_dense_groups_; }
  int dense_stride() const { return row_stride_; }
  const uint8_t* dense_bins() const { return bins_.data(); }
  const uint8_t* dense_row(data_size_t i) const { return bins_.data() + static_cast<size_t>(i) * row_stride_; }
  // multi-value sparse part (reference multi_val_sparse_bin.hpp, MI355X-first as one CSR of
  // global histogram bins): row i's non-zero sparse groups are sp_bins()[sp_ptr()[i] ..
  // sp_ptr()[i + 1]), each entry hist_start(group) + group bin, ascending
  bool has_sparse() const { return num_dense_groups_ < num_groups(); }
  const uint64_t* sp_ptr() const { return sp_ptr_.data(); }
  const uint32_t* sp_bins() const { return sp_bin_.data(); }
  size_t sparse_nnz() const { return sp_bin_.size(); }
  // every group packed row-major at row_stride() (device upload of a sparse-stored dataset)
  const uint8_t* RowsForDevice(std::vector<uint8_t>* scratch) const;
  void MaterializeRows(std::vector<uint8_t>* out) const;
  // sparse groups back into the dense matrix (AddFeaturesFrom, device packing)
  void Densify();
  static int FullStride(int ngroups, int width) {
    const int s = (ngroups * width + 3) / 4 * 4;
    return s == 0 ? 4 : s;
  }
  const FeatureInfo& feature(int inner) const { return features_[inner]; }
  const std::vector<FeatureInfo>& features() const { return features_; }
  const FeatureGroup& group(int g) const { return groups_[g]; }
  const std::vector<FeatureGroup>& groups() const { return groups_; }
  const BinMapper& mapper(int real_index) const { return mappers_[real_index]; }
  const BinMapper& inner_mapper(int inner) const { return mappers_[features_[inner].real_index]; }
  int InnerIndex(int real_index) const { return used_map_[real_index]; }
  const std::vector<std::string>& feature_names() const { return feature_names_; }
  void set_feature_names(const std::vector<std::string>& n);
  std::vector<std::string> feature_infos() const;
  Metadata& metadata() { return metadata_; }
  const Metadata& metadata() const { return metadata_; }
  const std::vector<int>& categorical_real() const { return categorical_; }
  // raw values of used features (kept only for linear_tree)
  bool has_raw() const { return !raw_.empty(); }
  double raw(data_size_t i, int inner) const { return raw_[static_cast<size_t>(i) * features_.size() + inner]; }
  // [num_data][num_features] raw values of the used features (linear_tree; empty otherwise)
  const std::vector<float>& raw_values() const { return raw_; }

  // Raw group bin of row i in group g.
  inline uint32_t GroupBin(data_size_t i, int g) const {
    if (g >= num_dense_groups_) return SparseGroupBin(i, g);
    const uint8_t* r = bins_.data() + static_cast<size_t>(i) * row_stride_;
    return bin_width_ == 1 ? r[g] : reinterpret_cast<const uint16_t*>(r)[g];
  }
  inline uint32_t SparseGroupBin(data_size_t i, int g) const {
    const uint32_t lo = static_cast<uint32_t>(groups_[g].hist_start);
    const uint32_t* b = sp_bin_.data() + sp_ptr_[i];
    const uint32_t* e = sp_bin_.data() + sp_ptr_[i + 1];
    const uint32_t* p = std::lower_bound(b, e, lo);
    return (p != e && *p < lo + static_cast<uint32_t>(groups_[g].num_bin)) ? *p - lo : 0u;
  }
  // Feature bin of row i for inner feature f (decoding the group bin).
  inline uint32_t FeatureBin(data_size_t i, int f) const {
    const FeatureInfo& fi = features_[f];
    uint32_t gb = GroupBin(i, fi.group);
    return DecodeBin(fi, gb);
  }
  static inline uint32_t DecodeBin(const FeatureInfo& fi, uint32_t gb) {
    int local = static_cast<int>(gb) - fi.offset;
    if (local < 0 || local >= fi.num_bin - 1) return fi.mfb;
    return static_cast<uint32_t>(local) < fi.mfb ? static_cast<uint32_t>(local) : static_cast<uint32_t>(local + 1);
  }
  static inline int EncodeBin(const FeatureInfo& fi, uint32_t b) {
    if (b == fi.mfb) return 0;
    return fi.offset + static_cast<int>(b) - (b > fi.mfb ? 1 : 0);
  }

  // Expand a packed group histogram (num_total_bin entries of (g,h)) into the
  // full per-feature histogram (num_bin entries), reconstructing the mfb bin.
  void FeatureHistogram(const double* group_hist, int f, double sum_g, double sum_h, double* out) const;

  // Streaming construction (LGBM_DatasetCreateByReference / PushRows).
  void InitEmptyLike(const Dataset& reference, data_size_t num_rows);
  void PushRows(const RowSource& src, data_size_t start_row);

  bool CheckAlign(const Dataset& other) const;
  // Adds columns of another dataset (LGBM_DatasetAddFeaturesFrom).
  void AddFeaturesFrom(const Dataset& other);
  std::string reference_key() const;  // identity of the binning (for valid-set checks)

 private:
  void BuildGroups(const Config& cfg, const std::vector<std::vector<int>>& sample_nonzero_rows,
                   data_size_t sample_cnt);
  void PackRows(const RowSource& src, data_size_t start_row = 0, bool reset = true);
  void FinalizeLayout();
  // moves groups whose rows are mostly at group bin 0 into the sparse CSR (sparse groups last)
  void CompressSparseGroups(double zero_threshold);

  data_size_t num_data_ = 0;
  int num_total_features_ = 0;
  std::vector<std::string> feature_names_;
  std::string parser_config_;
  std::vector<BinMapper> mappers_;  // per real feature
  std::vector<int> used_map_;       // real -> inner or -1
  std::vector<FeatureInfo> features_;
  std::vector<FeatureGroup> groups_;
  std::vector<int> categorical_;
  int num_total_bin_ = 0;
  int bin_width_ = 1;
  int row_stride_ = 0;            // stride of bins_ (dense groups only)
  int num_dense_groups_ = 0;
  std::vector<uint8_t> bins_;
  std::vector<uint64_t> sp_ptr_;  // num_data_ + 1 (empty: every group dense)
  std::vector<uint32_t> sp_bin_;
  std::vector<float> raw_;
  bool keep_raw_ = false;
  bool device_pack_ = false;  // device_type=gpu + device_binning: PackRows runs on the GPU
  Metadata metadata_;
  std::vector<int8_t> monotone_;
  std::vector<double> feature_penalty_;
};

// Dense row-major / column-major matrix source.
class DenseSource : public RowSource {
 public:
  DenseSource(const void* data, int dtype_f64, data_size_t nrow, int ncol, bool row_major)
      : data_(data), f64_(dtype_f64), nrow_(nrow), ncol_(ncol), row_major_(row_major) {}
  data_size_t num_rows() const override { return nrow_; }
  int num_cols() const override { return ncol_; }
  const void* data() const { return data_; }
  bool is_f64() const { return f64_ != 0; }
  bool row_major() const { return row_major_; }
  inline double At(data_size_t i, int j) const {
    size_t k = row_major_ ? static_cast<size_t>(i) * ncol_ + j : static_cast<size_t>(j) * nrow_ + i;
    return f64_ ? static_cast<const double*>(data_)[k] : static_cast<const float*>(data_)[k];
  }
  void GetRow(data_size_t i, std::vector<std::pair<int, double>>* out) const override {
    out->clear();
    for (int j = 0; j < ncol_; ++j) {
      double v = At(i, j);
      if (std::isnan(v) || std::fabs(v) > kZeroThreshold) out->emplace_back(j, v);
    }
  }

 private:
  const void* data_;
  int f64_;
  data_size_t nrow_;
  int ncol_;
  bool row_major_;
};

// CSR source (indptr int32/int64, indices int32, values f32/f64).
class CSRSource : public RowSource {
 public:
  CSRSource(const void* indptr, int indptr_i64, const int32_t* indices, const void* data, int data_f64,
            int64_t nindptr, int64_t nelem, int64_t ncol)
      : indptr_(indptr), i64_(indptr_i64), indices_(indices), data_(data), f64_(data_f64),
        nrow_(static_cast<data_size_t>(nindptr - 1)), ncol_(static_cast<int>(ncol)) { (void)nelem; }
  data_size_t num_rows() const override { return nrow_; }
  int num_cols() const override { return ncol_; }
  void GetRow(data_size_t i, std::vector<std::pair<int, double>>* out) const override {
    out->clear();
    int64_t b = i64_ ? static_cast<const int64_t*>(indptr_)[i] : static_cast<const int32_t*>(indptr_)[i];
    int64_t e = i64_ ? static_cast<const int64_t*>(indptr_)[i + 1] : static_cast<const int32_t*>(indptr_)[i + 1];
    for (int64_t k = b; k < e; ++k) {
      double v = f64_ ? static_cast<const double*>(data_)[k] : static_cast<const float*>(data_)[k];
      out->emplace_back(indices_[k], v);
    }
  }

 private:
  const void* indptr_;
  int i64_;
  const int32_t* indices_;
  const void* data_;
  int f64_;
  data_size_t nrow_;
  int ncol_;
};

// Owning row store used by the text loader and CSC conversion.
class OwnedSparseSource : public RowSource {
 public:
  std::vector<std::vector<std::pair<int, double>>> rows;
  int ncol = 0;
  data_size_t num_rows() const override { return static_cast<data_size_t>(rows.size()); }
  int num_cols() const override { return ncol; }
  void GetRow(data_size_t i, std::vector<std::pair<int, double>>* out) const override { *out = rows[i]; }
};

// Text file loading (CSV/TSV/LibSVM auto-detect; label/weight/group columns).
std::unique_ptr<Dataset> LoadDatasetFromFile(const std::string& filename, const Config& cfg,
                                             const Dataset* reference, int rank, int num_machines);
// Parses a text file into rows (used by prediction on files as well).
void ParseTextFile(const std::string& filename, bool header, int label_idx, OwnedSparseSource* rows,
                   std::vector<float>* labels, std::vector<std::string>* header_names, int* out_label_idx,
                   const std::vector<int>& ignore_cols, int weight_idx, std::vector<float>* weights,
                   int group_idx, std::vector<double>* group_ids);

}  // namespace lgap
