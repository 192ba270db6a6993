// coord_stress.cpp — native concurrency test of the coordinator (coord.cpp),
// meant to be built with ThreadSanitizer or AddressSanitizer+UBSan
// (tests/test_native_sanitizers.py).  SURVEY.md §5.2: the reference's job
// claim was update-then-find (task.lua:294-309) and could hand one job to two
// workers; here JOB_CLAIM is one atomic operation of the coordinator.  This
// program starts a coordinator in-process, inserts N jobs, lets T client
// threads (one TCP connection each) claim until none is left, and checks that
// every job was claimed exactly once; then T threads contend on a
// persistent-table lock (PT_LOCK / PT_UNLOCK) around a shared counter and the
// final count must equal the number of critical sections.
//
//   coord_stress [threads] [jobs]      exit 0 = ok
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" int mrc_start(const char* host, int port, const char* journal);

namespace {

struct Conn {
  int fd = -1;
  explicit Conn(int port) {
    fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(fd, (sockaddr*)&a, sizeof a) != 0) {
      perror("connect");
      exit(2);
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  }
  ~Conn() { close(fd); }
  void all(const void* p, size_t n, bool wr) {
    char* c = (char*)p;
    while (n) {
      ssize_t k = wr ? write(fd, c, n) : read(fd, c, n);
      if (k <= 0) {
        fprintf(stderr, "socket %s failed\n", wr ? "write" : "read");
        exit(2);
      }
      c += k;
      n -= (size_t)k;
    }
  }
  // request: u32 len | u16 op | fields (u32 len | bytes); response: u32 len | i32 status | fields
  int req(uint16_t op, const std::vector<std::string>& f, std::vector<std::string>* out = nullptr) {
    std::string body((const char*)&op, 2);
    for (auto& s : f) {
      uint32_t n = (uint32_t)s.size();
      body.append((const char*)&n, 4);
      body += s;
    }
    uint32_t n = (uint32_t)body.size();
    all(&n, 4, true);
    all(body.data(), body.size(), true);
    all(&n, 4, false);
    std::string resp(n, '\0');
    all(&resp[0], n, false);
    int32_t st;
    memcpy(&st, resp.data(), 4);
    if (out) {
      out->clear();
      for (size_t p = 4; p + 4 <= resp.size();) {
        uint32_t k;
        memcpy(&k, resp.data() + p, 4);
        out->push_back(resp.substr(p + 4, k));
        p += 4 + k;
      }
    }
    return st;
  }
};

enum : uint16_t { JOB_INSERT = 20, JOB_CLAIM = 24, PT_OPEN = 60, PT_LOCK = 62, PT_UNLOCK = 63 };

}  // namespace

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 8;
  const int N = argc > 2 ? atoi(argv[2]) : 2000;
  const int port = mrc_start("127.0.0.1", 0, "");
  if (port <= 0) {
    fprintf(stderr, "coordinator did not start\n");
    return 2;
  }
  {
    Conn c(port);
    for (int i = 0; i < N; ++i)
      if (c.req(JOB_INSERT, {"stress", "map_jobs", std::to_string(i), "{}", "0"}) != 0) {
        fprintf(stderr, "insert %d failed\n", i);
        return 1;
      }
  }
  // --- claims: every job exactly once
  std::vector<std::atomic<int>> seen(N);
  for (auto& s : seen) s = 0;
  std::atomic<int> claimed{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      Conn c(port);
      std::vector<std::string> out;
      const std::string worker = "w" + std::to_string(t);
      while (c.req(JOB_CLAIM, {"stress", "map_jobs", worker, worker + "-tmp", "1.0", "1"}, &out) == 0) {
        const int id = atoi(out.at(0).c_str());
        seen[id].fetch_add(1);
        claimed.fetch_add(1);
      }
    });
  for (auto& x : th) x.join();
  th.clear();
  int bad = 0;
  for (int i = 0; i < N; ++i) bad += seen[i].load() != 1;
  if (bad || claimed.load() != N) {
    fprintf(stderr, "claim check failed: %d jobs not claimed exactly once, %d claims for %d jobs\n", bad,
            claimed.load(), N);
    return 1;
  }
  // --- persistent-table lock: read-modify-write of one field under PT_LOCK
  {
    Conn c(port);
    c.req(PT_OPEN, {"stress", "singletons", "counter"});
  }
  const int K = 25;
  std::atomic<long> inside{0}, max_inside{0}, sections{0};
  for (int t = 0; t < T; ++t)
    th.emplace_back([&] {
      Conn c(port);
      std::vector<std::string> out;
      for (int k = 0; k < K; ++k) {
        // PT_LOCK sets the flag and returns whether it was already set
        while (c.req(PT_LOCK, {"stress", "singletons", "counter"}, &out) != 0 || atoi(out.at(0).c_str()) != 0)
          usleep(100);
        const long now = inside.fetch_add(1) + 1;
        long m = max_inside.load();
        while (now > m && !max_inside.compare_exchange_weak(m, now)) {
        }
        sections.fetch_add(1);
        inside.fetch_sub(1);
        c.req(PT_UNLOCK, {"stress", "singletons", "counter"});
      }
    });
  for (auto& x : th) x.join();
  if (max_inside.load() != 1 || sections.load() != (long)T * K) {
    fprintf(stderr, "lock check failed: max %ld holders at once, %ld sections\n", max_inside.load(),
            sections.load());
    return 1;
  }
  printf("coord_stress ok: %d threads, %d jobs claimed once each, %ld locked sections\n", T, N, sections.load());
  return 0;
}
