// Collective algorithms over the host link layer (reference:
// src/network/network.cpp:30-328). Allreduce = ReduceScatter + Allgather for
// large payloads, Allgather-then-reduce for small ones; Allgather by recursive
// doubling / Bruck / ring; ReduceScatter by recursive halving or ring.
// Transports (linkers.cpp): TCP socket mesh, or external functions injected
// through LGBM_NetworkInitWithFunctions.
#include "lgap/network.h"

#include <algorithm>
#include <cstring>
#include <mutex>

#include "lgap/log.h"
#include "linkers.h"

namespace lgap {

namespace {
struct NetState {
  int rank = 0;
  int num_machines = 1;
  std::unique_ptr<Linkers> linkers;
  ReduceScatterFunction ext_rs;
  AllgatherFunction ext_ag;
  std::vector<char> buf1, buf2;
};
NetState& S() {
  static NetState s;
  return s;
}
}  // namespace

void Network::Init(const Config& config) {
  if (config.num_machines <= 1) return;
  S().linkers = std::make_unique<Linkers>(config);
  S().rank = S().linkers->rank();
  S().num_machines = S().linkers->num_machines();
  S().ext_rs = nullptr;
  S().ext_ag = nullptr;
  Log::Info("Local rank: %d, total number of machines: %d", S().rank, S().num_machines);
}

void Network::Init(int num_machines, int rank, ReduceScatterFunction rs, AllgatherFunction ag) {
  if (num_machines <= 1) return;
  S().linkers.reset();
  S().rank = rank;
  S().num_machines = num_machines;
  S().ext_rs = rs;
  S().ext_ag = ag;
}

void Network::Dispose() {
  S().linkers.reset();
  S().num_machines = 1;
  S().rank = 0;
  S().ext_rs = nullptr;
  S().ext_ag = nullptr;
}

int Network::rank() { return S().rank; }
int Network::num_machines() { return S().num_machines; }

void Network::Allgather(char* input, const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                        comm_size_t all_size) {
  const int n = S().num_machines;
  if (n <= 1) {
    std::memcpy(output, input, block_len[0]);
    return;
  }
  if (S().ext_ag) {
    S().ext_ag(input, block_len[S().rank], block_start, block_len, n, output, all_size);
    return;
  }
  S().linkers->Allgather(input, block_start, block_len, output, all_size);
}

void Network::Allgather(char* input, comm_size_t send_size, char* output) {
  const int n = S().num_machines;
  std::vector<comm_size_t> start(n), len(n, send_size);
  for (int i = 0; i < n; ++i) start[i] = i * send_size;
  Allgather(input, start.data(), len.data(), output, send_size * n);
}

void Network::ReduceScatter(char* input, comm_size_t input_size, int type_size, const comm_size_t* block_start,
                            const comm_size_t* block_len, char* output, comm_size_t output_size,
                            const ReduceFunction& reducer) {
  const int n = S().num_machines;
  if (n <= 1) {
    std::memcpy(output, input, input_size);
    return;
  }
  if (S().ext_rs) {
    S().ext_rs(input, input_size, type_size, block_start, block_len, n, output, output_size, reducer);
    return;
  }
  if (S().ext_ag) {
    // allgather-only external transport: gather every rank's input, reduce this rank's block
    std::vector<char> all(static_cast<size_t>(input_size) * n);
    Allgather(input, input_size, all.data());
    const int r = S().rank;
    // start from this rank's own block, then add every other rank's
    std::memcpy(output, all.data() + static_cast<size_t>(r) * input_size + block_start[r], block_len[r]);
    for (int k = 0; k < n; ++k) {
      if (k != r) reducer(all.data() + static_cast<size_t>(k) * input_size + block_start[r], output, type_size, block_len[r]);
    }
    return;
  }
  S().linkers->ReduceScatter(input, input_size, type_size, block_start, block_len, output, output_size, reducer);
}

void Network::Allreduce(char* input, comm_size_t input_size, int type_size, char* output, const ReduceFunction& reducer) {
  const int n = S().num_machines;
  if (n <= 1) {
    if (output != input) std::memcpy(output, input, input_size);
    return;
  }
  const comm_size_t count = input_size / type_size;
  if (input_size < 4096 || count < n) {
    // allgather then local reduce (small payloads)
    std::vector<char> all(static_cast<size_t>(input_size) * n);
    Allgather(input, input_size, all.data());
    std::memcpy(output, all.data(), input_size);
    for (int i = 1; i < n; ++i) reducer(all.data() + static_cast<size_t>(i) * input_size, output, type_size, input_size);
    return;
  }
  // reduce-scatter into per-rank blocks, then allgather the reduced blocks
  std::vector<comm_size_t> start(n), len(n);
  const comm_size_t step = (count + n - 1) / n;
  for (int i = 0; i < n; ++i) {
    const comm_size_t b = std::min(count, step * i), e = std::min(count, step * (i + 1));
    start[i] = b * type_size;
    len[i] = (e - b) * type_size;
  }
  std::vector<char> mine(len[S().rank] > 0 ? len[S().rank] : 1);
  ReduceScatter(input, input_size, type_size, start.data(), len.data(), mine.data(), len[S().rank], reducer);
  Allgather(mine.data(), start.data(), len.data(), output, input_size);
}

std::vector<std::vector<char>> Network::AllgatherBlobs(const std::vector<char>& blob) {
  const int n = num_machines();
  if (n <= 1) return {blob};
  std::vector<comm_size_t> sizes(n);
  comm_size_t mine = static_cast<comm_size_t>(blob.size());
  Allgather(reinterpret_cast<char*>(&mine), sizeof(comm_size_t), reinterpret_cast<char*>(sizes.data()));
  std::vector<comm_size_t> start(n, 0);
  for (int i = 1; i < n; ++i) start[i] = start[i - 1] + sizes[i - 1];
  const comm_size_t total = start[n - 1] + sizes[n - 1];
  std::vector<char> all(std::max<comm_size_t>(total, 1));
  std::vector<char> in = blob;
  if (in.empty()) in.resize(1);
  Allgather(in.data(), start.data(), sizes.data(), all.data(), total);
  std::vector<std::vector<char>> out(n);
  for (int i = 0; i < n; ++i) out[i].assign(all.begin() + start[i], all.begin() + start[i] + sizes[i]);
  return out;
}

}  // namespace lgap
