// Arrow C data interface reader (see include/lgap/arrow.h).
#include "lgap/arrow.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#include "lgap/log.h"

namespace lgap {

namespace {

char FormatType(const char* fmt) {
  if (fmt == nullptr || fmt[0] == '\0' || fmt[1] != '\0') {
    Log::Fatal("Unsupported Arrow column format '%s' (numeric and boolean columns only)", fmt ? fmt : "");
  }
  switch (fmt[0]) {
    case 'c': case 'C': case 's': case 'S': case 'i': case 'I': case 'l': case 'L': case 'f': case 'g': case 'b':
      return fmt[0];
    default:
      Log::Fatal("Unsupported Arrow column format '%s' (numeric and boolean columns only)", fmt);
  }
  return 'g';
}

inline bool BitSet(const uint8_t* bits, int64_t i) { return (bits[i >> 3] >> (i & 7)) & 1; }

}  // namespace

double ArrowColumnChunk::Get(int64_t i) const {
  const int64_t k = offset + i;
  if (validity != nullptr && !BitSet(validity, k)) return std::numeric_limits<double>::quiet_NaN();
  switch (type) {
    case 'c': return static_cast<const int8_t*>(values)[k];
    case 'C': return static_cast<const uint8_t*>(values)[k];
    case 's': return static_cast<const int16_t*>(values)[k];
    case 'S': return static_cast<const uint16_t*>(values)[k];
    case 'i': return static_cast<const int32_t*>(values)[k];
    case 'I': return static_cast<const uint32_t*>(values)[k];
    case 'l': return static_cast<double>(static_cast<const int64_t*>(values)[k]);
    case 'L': return static_cast<double>(static_cast<const uint64_t*>(values)[k]);
    case 'f': return static_cast<const float*>(values)[k];
    case 'g': return static_cast<const double*>(values)[k];
    case 'b': return BitSet(static_cast<const uint8_t*>(values), k) ? 1.0 : 0.0;
    default: return std::numeric_limits<double>::quiet_NaN();
  }
}

ArrowTable::ArrowTable(int64_t n_chunks, const ArrowArray* chunks, const ArrowSchema* schema) {
  if (schema == nullptr || schema->format == nullptr) Log::Fatal("Arrow schema is missing");
  // a struct schema (record batch) holds one child per column; a bare primitive
  // schema is a single column
  const bool is_struct = std::strcmp(schema->format, "+s") == 0;
  std::vector<const ArrowSchema*> col_schemas;
  if (is_struct) {
    for (int64_t c = 0; c < schema->n_children; ++c) col_schemas.push_back(schema->children[c]);
  } else {
    col_schemas.push_back(schema);
  }
  for (size_t c = 0; c < col_schemas.size(); ++c) {
    const char* nm = col_schemas[c]->name;
    names_.push_back(nm && nm[0] ? nm : "Column_" + std::to_string(c));
  }
  starts_.push_back(0);
  for (int64_t k = 0; k < n_chunks; ++k) {
    const ArrowArray& batch = chunks[k];
    std::vector<ArrowColumnChunk> cc;
    for (size_t c = 0; c < col_schemas.size(); ++c) {
      const ArrowArray* col = is_struct ? batch.children[c] : &batch;
      if (col->n_buffers < 2) Log::Fatal("Arrow column %zu: expected validity + values buffers", c);
      ArrowColumnChunk ch;
      ch.type = FormatType(col_schemas[c]->format);
      // a struct array's own offset shifts every child
      ch.offset = col->offset + (is_struct ? batch.offset : 0);
      ch.length = batch.length;
      ch.validity = col->null_count == 0 ? nullptr : static_cast<const uint8_t*>(col->buffers[0]);
      ch.values = col->buffers[1];
      cc.push_back(ch);
    }
    cols_.push_back(std::move(cc));
    num_rows_ += batch.length;
    starts_.push_back(num_rows_);
  }
}

double ArrowTable::At(int64_t row, int col) const {
  const size_t k = std::upper_bound(starts_.begin(), starts_.end(), row) - starts_.begin() - 1;
  return cols_[k][col].Get(row - starts_[k]);
}

std::vector<double> ArrowTable::Column(int col) const {
  std::vector<double> out(static_cast<size_t>(num_rows_));
  for (size_t k = 0; k < cols_.size(); ++k) {
    const ArrowColumnChunk& ch = cols_[k][col];
    for (int64_t i = 0; i < ch.length; ++i) out[starts_[k] + i] = ch.Get(i);
  }
  return out;
}

void ArrowSource::GetRow(data_size_t i, std::vector<std::pair<int, double>>* out) const {
  out->clear();
  for (int j = 0; j < t_.num_columns(); ++j) {
    const double v = t_.At(i, j);
    if (std::isnan(v) || std::fabs(v) > kZeroThreshold) out->emplace_back(j, v);
  }
}

}  // namespace lgap
