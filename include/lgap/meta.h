// Core scalar types and constants shared by host C++ and HIP device code.
// Semantics follow the reference (include/LightGBM/meta.h:18-91): 32-bit row
// indices, float scores/labels, double histogram accumulators.
#pragma once

#include <cstdint>
#include <cstddef>
#include <limits>
#include <functional>
#include <vector>

#if defined(__HIPCC__)
#define LGAP_HD __host__ __device__
#define LGAP_D __device__
#else
#define LGAP_HD
#define LGAP_D
#endif

namespace lgap {

using data_size_t = int32_t;
using score_t = float;
using label_t = float;
using hist_t = double;
using comm_size_t = int32_t;

constexpr double kEpsilon = 1e-15;
constexpr double kZeroThreshold = 1e-35f;
constexpr double kMinScore = -std::numeric_limits<double>::infinity();
constexpr double kMaxScore = std::numeric_limits<double>::infinity();
constexpr double kSparseThreshold = 0.7;
constexpr int kMaxTreeOutput = 100;
constexpr const char* kModelVersion = "v4";

// Reducer signature used by the host collective layer (meta.h ReduceFunction).
using ReduceFunction = std::function<void(const char* src, char* dst, int type_size, comm_size_t len)>;
using ReduceScatterFunction = std::function<void(char* input, comm_size_t input_size, int type_size,
                                                 const comm_size_t* block_start, const comm_size_t* block_len,
                                                 int num_block, char* output, comm_size_t output_size,
                                                 const ReduceFunction& reducer)>;
using AllgatherFunction = std::function<void(char* input, comm_size_t input_size, const comm_size_t* block_start,
                                             const comm_size_t* block_len, int num_block, char* output,
                                             comm_size_t output_size)>;

enum class MissingType : int8_t { None = 0, Zero = 1, NaN = 2 };
enum class BinType : int8_t { Numerical = 0, Categorical = 1 };

}  // namespace lgap
