// Arrow C data interface consumer (reference include/LightGBM/arrow.h,
// arrow.tpp): record batches exported by any Arrow producer (pyarrow's
// RecordBatch._export_to_c, arrow-rs, ...) are read in place, column by column,
// without an Arrow library dependency. Nulls are missing values (NaN).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "lgap/dataset.h"

extern "C" {
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
struct ArrowSchema {
  const char* format;
  const char* name;
  const char* metadata;
  int64_t flags;
  int64_t n_children;
  struct ArrowSchema** children;
  struct ArrowSchema* dictionary;
  void (*release)(struct ArrowSchema*);
  void* private_data;
};

struct ArrowArray {
  int64_t length;
  int64_t null_count;
  int64_t offset;
  int64_t n_buffers;
  int64_t n_children;
  const void** buffers;
  struct ArrowArray** children;
  struct ArrowArray* dictionary;
  void (*release)(struct ArrowArray*);
  void* private_data;
};
#endif
}

namespace lgap {

// One primitive column chunk: validity bitmap + values, typed by its format.
struct ArrowColumnChunk {
  char type = 'g';  // Arrow format char: c C s S i I l L f g b
  int64_t offset = 0;
  int64_t length = 0;
  const uint8_t* validity = nullptr;
  const void* values = nullptr;
  double Get(int64_t i) const;  // i local to the chunk; NaN for null
};

// A chunked table: `n_chunks` struct arrays (record batches) sharing `schema`.
class ArrowTable {
 public:
  ArrowTable(int64_t n_chunks, const ArrowArray* chunks, const ArrowSchema* schema);
  int64_t num_rows() const { return num_rows_; }
  int num_columns() const { return static_cast<int>(names_.size()); }
  const std::vector<std::string>& names() const { return names_; }
  double At(int64_t row, int col) const;
  // one column as doubles (for label / weight / init_score / group fields)
  std::vector<double> Column(int col) const;

 private:
  std::vector<std::string> names_;
  std::vector<int64_t> starts_;                      // chunk start rows (+ total)
  std::vector<std::vector<ArrowColumnChunk>> cols_;  // [chunk][col]
  int64_t num_rows_ = 0;
};

// RowSource over an ArrowTable for the dataset builder / predictor.
class ArrowSource : public RowSource {
 public:
  explicit ArrowSource(const ArrowTable& t) : t_(t) {}
  data_size_t num_rows() const override { return static_cast<data_size_t>(t_.num_rows()); }
  int num_cols() const override { return t_.num_columns(); }
  void GetRow(data_size_t i, std::vector<std::pair<int, double>>* out) const override;

 private:
  const ArrowTable& t_;
};

}  // namespace lgap
