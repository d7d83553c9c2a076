// TCP full-mesh link layer (reference: src/network/linkers.h,
// linkers_socket.cpp, socket_wrapper.hpp): machine list parsing
// ("ip port" / "ip:port" lines or the `machines` string), lower rank connects
// to higher rank with exponential backoff, TCP_NODELAY, receive timeout of
// `time_out` minutes, and ring / recursive-doubling / Bruck Allgather and ring /
// recursive-halving ReduceScatter over the mesh.
#pragma once

#include <string>
#include <vector>

#include "lgap/config.h"
#include "lgap/meta.h"

namespace lgap {

class Linkers {
 public:
  explicit Linkers(const Config& config);
  ~Linkers();
  int rank() const { return rank_; }
  int num_machines() const { return num_machines_; }

  void Send(int peer, const char* data, size_t len);
  void Recv(int peer, char* data, size_t len);
  void SendRecv(int send_peer, const char* send_data, size_t send_len, int recv_peer, char* recv_data, size_t recv_len);

  void Allgather(char* input, const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                 comm_size_t all_size);
  void ReduceScatter(char* input, comm_size_t input_size, int type_size, const comm_size_t* block_start,
                     const comm_size_t* block_len, char* output, comm_size_t output_size, const ReduceFunction& reducer);
  double network_seconds() const { return net_time_; }

 private:
  void AllgatherRing(const comm_size_t* start, const comm_size_t* len, char* output);
  void AllgatherRecursiveDoubling(const comm_size_t* start, const comm_size_t* len, char* output);
  void AllgatherBruck(const comm_size_t* start, const comm_size_t* len, char* output);
  void ReduceScatterRing(char* input, comm_size_t input_size, int type_size, const comm_size_t* start,
                         const comm_size_t* len, char* output, const ReduceFunction& reducer);
  void ReduceScatterRecursiveHalving(char* input, comm_size_t input_size, int type_size, const comm_size_t* start,
                                     const comm_size_t* len, char* output, const ReduceFunction& reducer);
  void ParseMachines(const Config& config);
  void Construct(int listen_port, int time_out_min);
  int rank_ = 0;
  int num_machines_ = 1;
  std::vector<std::string> ips_;
  std::vector<int> ports_;
  std::vector<int> socks_;
  int listen_sock_ = -1;
  double net_time_ = 0.0;
};

}  // namespace lgap
