// Host collective layer (reference: include/LightGBM/network.h:22-313,
// src/network/network.cpp). Used by the CPU parallel learners, distributed
// bin finding and the scalar syncs of objectives. Transports: a TCP socket
// mesh (machines list), or externally injected reduce-scatter/allgather
// functions (LGBM_NetworkInitWithFunctions). Device learners exchange
// histograms over RCCL (see device/comm) instead of through this layer.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "lgap/config.h"
#include "lgap/meta.h"

namespace lgap {

class Linkers;

class Network {
 public:
  static void Init(const Config& config);
  static void Init(int num_machines, int rank, ReduceScatterFunction rs, AllgatherFunction ag);
  static void Dispose();
  static int rank();
  static int num_machines();

  // Generic collectives over raw bytes.
  static void Allreduce(char* input, comm_size_t input_size, int type_size, char* output, const ReduceFunction& reducer);
  static void Allgather(char* input, comm_size_t send_size, char* output);
  static void Allgather(char* input, const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                        comm_size_t all_size);
  static void ReduceScatter(char* input, comm_size_t input_size, int type_size, const comm_size_t* block_start,
                            const comm_size_t* block_len, char* output, comm_size_t output_size,
                            const ReduceFunction& reducer);

  template <typename T>
  static T GlobalSyncUpBySum(T v) {
    if (num_machines() <= 1) return v;
    T out = v;
    Allreduce(reinterpret_cast<char*>(&v), sizeof(T), sizeof(T), reinterpret_cast<char*>(&out), SumReducer<T>());
    return out;
  }
  template <typename T>
  static T GlobalSyncUpByMax(T v) {
    if (num_machines() <= 1) return v;
    T out = v;
    Allreduce(reinterpret_cast<char*>(&v), sizeof(T), sizeof(T), reinterpret_cast<char*>(&out), MaxReducer<T>());
    return out;
  }
  template <typename T>
  static T GlobalSyncUpByMin(T v) {
    if (num_machines() <= 1) return v;
    T out = v;
    Allreduce(reinterpret_cast<char*>(&v), sizeof(T), sizeof(T), reinterpret_cast<char*>(&out), MinReducer<T>());
    return out;
  }
  template <typename T>
  static T GlobalSyncUpByMean(T v) {
    if (num_machines() <= 1) return v;
    return GlobalSyncUpBySum(v) / static_cast<T>(num_machines());
  }
  template <typename T>
  static void GlobalSum(std::vector<T>* v) {
    if (num_machines() <= 1 || v->empty()) return;
    std::vector<T> out(v->size());
    Allreduce(reinterpret_cast<char*>(v->data()), static_cast<comm_size_t>(sizeof(T) * v->size()), sizeof(T),
              reinterpret_cast<char*>(out.data()), SumReducer<T>());
    *v = out;
  }
  // Gathers one variable-length byte blob per rank.
  static std::vector<std::vector<char>> AllgatherBlobs(const std::vector<char>& mine);

  template <typename T>
  static ReduceFunction SumReducer() {
    return [](const char* src, char* dst, int type_size, comm_size_t len) {
      for (comm_size_t i = 0; i < len; i += type_size) {
        *reinterpret_cast<T*>(dst + i) += *reinterpret_cast<const T*>(src + i);
      }
    };
  }
  template <typename T>
  static ReduceFunction MaxReducer() {
    return [](const char* src, char* dst, int type_size, comm_size_t len) {
      for (comm_size_t i = 0; i < len; i += type_size) {
        T& d = *reinterpret_cast<T*>(dst + i);
        const T s = *reinterpret_cast<const T*>(src + i);
        if (s > d) d = s;
      }
    };
  }
  template <typename T>
  static ReduceFunction MinReducer() {
    return [](const char* src, char* dst, int type_size, comm_size_t len) {
      for (comm_size_t i = 0; i < len; i += type_size) {
        T& d = *reinterpret_cast<T*>(dst + i);
        const T s = *reinterpret_cast<const T*>(src + i);
        if (s < d) d = s;
      }
    };
  }
};

}  // namespace lgap
