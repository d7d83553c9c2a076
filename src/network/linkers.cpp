#include "linkers.h"

#include <arpa/inet.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <fstream>
#include <set>
#include <thread>

#include "lgap/common.h"
#include "lgap/log.h"

namespace lgap {

namespace {
std::set<std::string> LocalIPs() {
  std::set<std::string> out = {"127.0.0.1", "localhost"};
  struct ifaddrs* ifs = nullptr;
  if (getifaddrs(&ifs) == 0) {
    for (auto* p = ifs; p != nullptr; p = p->ifa_next) {
      if (p->ifa_addr && p->ifa_addr->sa_family == AF_INET) {
        char buf[INET_ADDRSTRLEN];
        inet_ntop(AF_INET, &reinterpret_cast<sockaddr_in*>(p->ifa_addr)->sin_addr, buf, sizeof(buf));
        out.insert(buf);
      }
    }
    freeifaddrs(ifs);
  }
  return out;
}

void SendAll(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) Log::Fatal("Socket send failed: %s", strerror(errno));
    p += k;
    n -= static_cast<size_t>(k);
  }
}
void RecvAll(int fd, char* p, size_t n) {
  while (n > 0) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) Log::Fatal("Socket recv failed (peer closed or timeout): %s", strerror(errno));
    p += k;
    n -= static_cast<size_t>(k);
  }
}
}  // namespace

void Linkers::ParseMachines(const Config& config) {
  std::vector<std::string> lines;
  if (!config.machines.empty()) {
    lines = common::Split(config.machines, ',');
  } else if (!config.machine_list_filename.empty()) {
    std::ifstream in(config.machine_list_filename);
    if (!in) Log::Fatal("Cannot open machine list file %s", config.machine_list_filename.c_str());
    std::string l;
    while (std::getline(in, l)) {
      l = common::Trim(l);
      if (!l.empty() && l[0] != '#') lines.push_back(l);
    }
  } else {
    Log::Fatal("Machine list is required for distributed training (machines or machine_list_filename)");
  }
  for (auto& l : lines) {
    auto toks = common::SplitAny(l, " \t:");
    if (toks.size() < 2) Log::Fatal("Wrong machine list entry: %s", l.c_str());
    ips_.push_back(toks[0]);
    ports_.push_back(common::AtoiOrDie(toks[1]));
  }
  num_machines_ = static_cast<int>(ips_.size());
  if (num_machines_ != config.num_machines) {
    Log::Warning("num_machines (%d) differs from the machine list size (%d); using the list", config.num_machines,
                 num_machines_);
  }
  auto local = LocalIPs();
  rank_ = -1;
  for (int i = 0; i < num_machines_; ++i) {
    if (local.count(ips_[i]) && ports_[i] == config.local_listen_port) {
      rank_ = i;
      break;
    }
  }
  if (rank_ < 0) Log::Fatal("Machine list does not contain the local machine (port %d)", config.local_listen_port);
}

Linkers::Linkers(const Config& config) {
  ParseMachines(config);
  Construct(ports_[rank_], config.time_out);
}

void Linkers::Construct(int listen_port, int time_out_min) {
  socks_.assign(num_machines_, -1);
  listen_sock_ = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(listen_sock_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  addr.sin_port = htons(static_cast<uint16_t>(listen_port));
  if (::bind(listen_sock_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
    Log::Fatal("Binding port %d failed: %s", listen_port, strerror(errno));
  }
  ::listen(listen_sock_, num_machines_);
  // accept from lower ranks in a helper thread while connecting to higher ranks
  std::thread acceptor([&] {
    for (int k = 0; k < rank_; ++k) {
      int fd = ::accept(listen_sock_, nullptr, nullptr);
      if (fd < 0) Log::Fatal("Accept failed: %s", strerror(errno));
      int peer;
      RecvAll(fd, reinterpret_cast<char*>(&peer), sizeof(peer));
      socks_[peer] = fd;
    }
  });
  for (int j = rank_ + 1; j < num_machines_; ++j) {
    int delay_ms = 200;
    int fd = -1;
    for (int attempt = 0; attempt < 20; ++attempt) {
      fd = ::socket(AF_INET, SOCK_STREAM, 0);
      sockaddr_in pa{};
      pa.sin_family = AF_INET;
      pa.sin_port = htons(static_cast<uint16_t>(ports_[j]));
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      if (getaddrinfo(ips_[j].c_str(), nullptr, &hints, &res) == 0 && res) {
        pa.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
        freeaddrinfo(res);
      } else {
        inet_pton(AF_INET, ips_[j].c_str(), &pa.sin_addr);
      }
      if (::connect(fd, reinterpret_cast<sockaddr*>(&pa), sizeof(pa)) == 0) break;
      ::close(fd);
      fd = -1;
      std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms));
      delay_ms = static_cast<int>(delay_ms * 1.3);
    }
    if (fd < 0) Log::Fatal("Connecting to rank %d (%s:%d) failed", j, ips_[j].c_str(), ports_[j]);
    SendAll(fd, reinterpret_cast<const char*>(&rank_), sizeof(rank_));
    socks_[j] = fd;
  }
  acceptor.join();
  timeval tv{};
  tv.tv_sec = static_cast<long>(time_out_min) * 60;
  for (int i = 0; i < num_machines_; ++i) {
    if (i == rank_) continue;
    int one2 = 1;
    setsockopt(socks_[i], IPPROTO_TCP, TCP_NODELAY, &one2, sizeof(one2));
    int bufsz = 1 << 20;
    setsockopt(socks_[i], SOL_SOCKET, SO_SNDBUF, &bufsz, sizeof(bufsz));
    setsockopt(socks_[i], SOL_SOCKET, SO_RCVBUF, &bufsz, sizeof(bufsz));
    setsockopt(socks_[i], SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  }
  Log::Info("Connected to %d machines", num_machines_ - 1);
}

Linkers::~Linkers() {
  for (int fd : socks_) if (fd >= 0) ::close(fd);
  if (listen_sock_ >= 0) ::close(listen_sock_);
  if (net_time_ > 0) Log::Debug("Network time: %f seconds", net_time_);
}

void Linkers::Send(int peer, const char* data, size_t len) { SendAll(socks_[peer], data, len); }
void Linkers::Recv(int peer, char* data, size_t len) { RecvAll(socks_[peer], data, len); }

void Linkers::SendRecv(int sp, const char* sd, size_t sl, int rp, char* rd, size_t rl) {
  auto t0 = std::chrono::steady_clock::now();
  if (sl <= 64 * 1024) {
    Send(sp, sd, sl);
    Recv(rp, rd, rl);
  } else {
    std::thread th([&] { Send(sp, sd, sl); });
    Recv(rp, rd, rl);
    th.join();
  }
  net_time_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// ---------------------------------------------------------------------------
// Collectives over the mesh (reference src/network/network.cpp:150-328):
//   Allgather     ring for large payloads (>= 10 MB, < 64 ranks), recursive
//                 doubling for power-of-two rank counts, Bruck otherwise;
//   ReduceScatter recursive halving for power-of-two rank counts with
//                 contiguous ascending blocks, ring otherwise.
namespace {
bool IsPow2(int n) { return n > 0 && (n & (n - 1)) == 0; }
bool Ascending(const comm_size_t* start, const comm_size_t* len, int n) {
  for (int i = 1; i < n; ++i) {
    if (start[i] != start[i - 1] + len[i - 1]) return false;
  }
  return true;
}
constexpr comm_size_t kRingThreshold = 10 * 1024 * 1024;
}  // namespace

void Linkers::Allgather(char* input, const comm_size_t* start, const comm_size_t* len, char* output,
                        comm_size_t all_size) {
  const int n = num_machines_;
  std::memcpy(output + start[rank_], input, len[rank_]);
  const bool contiguous = Ascending(start, len, n);
  if (all_size >= kRingThreshold && n < 64) {
    AllgatherRing(start, len, output);
  } else if (IsPow2(n) && contiguous) {
    AllgatherRecursiveDoubling(start, len, output);
  } else {
    AllgatherBruck(start, len, output);
  }
}

void Linkers::AllgatherRing(const comm_size_t* start, const comm_size_t* len, char* output) {
  const int n = num_machines_;
  const int next = (rank_ + 1) % n, prev = (rank_ - 1 + n) % n;
  for (int s = 0; s < n - 1; ++s) {
    const int sb = (rank_ - s + n) % n;
    const int rb = (rank_ - s - 1 + n) % n;
    SendRecv(next, output + start[sb], len[sb], prev, output + start[rb], len[rb]);
  }
}

// log2(n) steps; at distance d each rank swaps its gathered run of d blocks with rank ^ d
void Linkers::AllgatherRecursiveDoubling(const comm_size_t* start, const comm_size_t* len, char* output) {
  const int n = num_machines_;
  for (int d = 1; d < n; d <<= 1) {
    const int peer = rank_ ^ d;
    const int mine = rank_ & ~(d - 1), theirs = peer & ~(d - 1);
    const comm_size_t sb = start[mine], rb = start[theirs];
    const comm_size_t sl = start[mine + d - 1] + len[mine + d - 1] - sb;
    const comm_size_t rl = start[theirs + d - 1] + len[theirs + d - 1] - rb;
    SendRecv(peer, output + sb, sl, peer, output + rb, rl);
  }
}

// ceil(log2(n)) steps for any n: blocks are held in rank-relative order
// (slot j = rank + j); at distance d the first min(d, n - d) slots go to rank - d
void Linkers::AllgatherBruck(const comm_size_t* start, const comm_size_t* len, char* output) {
  const int n = num_machines_;
  std::vector<char> rel;
  std::vector<comm_size_t> roff(n + 1, 0);
  for (int j = 0; j < n; ++j) roff[j + 1] = roff[j] + len[(rank_ + j) % n];
  rel.resize(std::max<comm_size_t>(roff[n], 1));
  std::memcpy(rel.data(), output + start[rank_], len[rank_]);
  for (int d = 1; d < n; d <<= 1) {
    const int cnt = std::min(d, n - d);
    const int to = (rank_ - d + n) % n, from = (rank_ + d) % n;
    // the receiver's slots [d, d + cnt) are the sender's [0, cnt): sizes from the sender's view
    comm_size_t recv_bytes = 0;
    for (int j = 0; j < cnt; ++j) recv_bytes += len[(from + j) % n];
    SendRecv(to, rel.data(), roff[cnt], from, rel.data() + roff[d], recv_bytes);
  }
  for (int j = 1; j < n; ++j) {
    const int r = (rank_ + j) % n;
    std::memcpy(output + start[r], rel.data() + roff[j], len[r]);
  }
}

void Linkers::ReduceScatter(char* input, comm_size_t input_size, int type_size, const comm_size_t* start,
                            const comm_size_t* len, char* output, comm_size_t output_size,
                            const ReduceFunction& reducer) {
  const int n = num_machines_;
  if (IsPow2(n) && Ascending(start, len, n)) {
    ReduceScatterRecursiveHalving(input, input_size, type_size, start, len, output, reducer);
  } else {
    ReduceScatterRing(input, input_size, type_size, start, len, output, reducer);
  }
  (void)output_size;
}

void Linkers::ReduceScatterRing(char* input, comm_size_t input_size, int type_size, const comm_size_t* start,
                                const comm_size_t* len, char* output, const ReduceFunction& reducer) {
  const int n = num_machines_;
  std::vector<char> acc(input, input + input_size);
  const int next = (rank_ + 1) % n, prev = (rank_ - 1 + n) % n;
  std::vector<char> tmp;
  for (int s = 0; s < n - 1; ++s) {
    const int sb = (rank_ - s - 1 + 2 * n) % n;
    const int rb = (rank_ - s - 2 + 2 * n) % n;
    tmp.resize(len[rb] > 0 ? len[rb] : 1);
    SendRecv(next, acc.data() + start[sb], len[sb], prev, tmp.data(), len[rb]);
    if (len[rb] > 0) reducer(tmp.data(), acc.data() + start[rb], type_size, len[rb]);
  }
  std::memcpy(output, acc.data() + start[rank_], len[rank_]);
}

// log2(n) steps: the live rank range halves each step; the half that holds the
// partner's blocks is sent, the own half is received and reduced in place
void Linkers::ReduceScatterRecursiveHalving(char* input, comm_size_t input_size, int type_size,
                                            const comm_size_t* start, const comm_size_t* len, char* output,
                                            const ReduceFunction& reducer) {
  const int n = num_machines_;
  std::vector<char> acc(input, input + input_size);
  std::vector<char> tmp;
  int lo = 0, hi = n;
  for (int d = n / 2; d >= 1; d >>= 1) {
    const int mid = lo + d;
    const bool upper = rank_ >= mid;
    const int peer = upper ? rank_ - d : rank_ + d;
    const int keep_lo = upper ? mid : lo, keep_hi = upper ? hi : mid;
    const int give_lo = upper ? lo : mid, give_hi = upper ? mid : hi;
    const comm_size_t kb = start[keep_lo], kl = start[keep_hi - 1] + len[keep_hi - 1] - kb;
    const comm_size_t gb = start[give_lo], gl = start[give_hi - 1] + len[give_hi - 1] - gb;
    tmp.resize(std::max<comm_size_t>(kl, 1));
    SendRecv(peer, acc.data() + gb, gl, peer, tmp.data(), kl);
    if (kl > 0) reducer(tmp.data(), acc.data() + kb, type_size, kl);
    lo = keep_lo;
    hi = keep_hi;
  }
  std::memcpy(output, acc.data() + start[rank_], len[rank_]);
}

}  // namespace lgap
