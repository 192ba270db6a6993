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

enum : uint16_t {
  JOB_INSERT = 20, JOB_CLAIM = 24, JOB_CLAIM_WAIT = 31, BLOB_PUT_MANY = 54, BLOB_GET_MANY = 55, BLOB_DEL_MANY = 56,
  PT_OPEN = 60, PT_LOCK = 62, PT_UNLOCK = 63
};

// A blob body whose every byte is a function of (writer, version): a reader
// can tell a torn or mixed body from an intact one.
std::string body_of(int t, int k, size_t n) {
  std::string b(n, '\0');
  for (size_t i = 0; i < n; ++i) b[i] = (char)((t * 131 + k * 7 + (int)(i % 251)) & 0xFF);
  b.replace(0, 8, std::to_string(1000 + t).substr(0, 4) + std::to_string(1000 + k % 9000).substr(0, 4));
  return b;
}

bool intact(const std::string& b) {
  if (b.size() < 8) return false;
  const int t = atoi(b.substr(0, 4).c_str()) - 1000, k = atoi(b.substr(4, 4).c_str()) - 1000;
  return b == body_of(t, k, b.size());
}

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
  th.clear();
  if (max_inside.load() != 1 || sections.load() != (long)T * K) {
    fprintf(stderr, "lock check failed: max %ld holders at once, %ld sections\n", max_inside.load(),
            sections.load());
    return 1;
  }
  // --- blobs: concurrent batched puts / gets / deletes of 64 KiB bodies, one
  // name shared by every thread (its body must always be one writer's intact
  // version: bodies are swapped in whole, never copied under a reader)
  std::atomic<int> blob_bad{0};
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      Conn c(port);
      std::vector<std::string> out;
      for (int k = 0; k < 60; ++k) {
        const std::string own = "own." + std::to_string(t) + "." + std::to_string(k);
        const std::string mine = body_of(t, k, 65536);
        c.req(BLOB_PUT_MANY, {"stress", own, mine, "shared", body_of(t, k, 32768 + 4096 * (k % 8))});
        if (c.req(BLOB_GET_MANY, {"stress", own, "shared"}, &out) != 0 || out.size() != 4 || out[0] != "1" ||
            out[1] != mine || out[2] != "1" || !intact(out[3]))
          blob_bad.fetch_add(1);
        if (k % 3 == 2) c.req(BLOB_DEL_MANY, {"stress", own});
      }
    });
  for (auto& x : th) x.join();
  th.clear();
  if (blob_bad.load()) {
    fprintf(stderr, "blob check failed: %d bad reads\n", blob_bad.load());
    return 1;
  }
  // --- long-poll claims: claimers block in JOB_CLAIM_WAIT while one thread
  // inserts jobs one at a time; every job is claimed exactly once and the
  // claimers return once the inserter is done and the queue stays empty
  const int N2 = 400;
  std::vector<std::atomic<int>> seen2(N2);
  for (auto& x : seen2) x = 0;
  std::atomic<bool> inserting{true};
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      Conn c(port);
      std::vector<std::string> out;
      const std::string worker = "lp" + std::to_string(t);
      for (;;) {
        const int st = c.req(JOB_CLAIM_WAIT, {"stress", "50", "lp_jobs", worker, worker + "-tmp", "1.0", "1"}, &out);
        if (st == 0) {
          seen2[atoi(out.at(0).c_str())].fetch_add(1);
        } else if (!inserting.load()) {
          break;
        }
      }
    });
  {
    Conn c(port);
    for (int i = 0; i < N2; ++i) {
      c.req(JOB_INSERT, {"stress", "lp_jobs", std::to_string(i), "{}", "0"});
      if (i % 50 == 0) usleep(2000);
    }
    usleep(100000);  // every job claimable before the claimers may stop
    inserting = false;
  }
  for (auto& x : th) x.join();
  int bad2 = 0;
  for (int i = 0; i < N2; ++i) bad2 += seen2[i].load() != 1;
  if (bad2) {
    fprintf(stderr, "long-poll claim check failed: %d jobs not claimed exactly once\n", bad2);
    return 1;
  }
  printf("coord_stress ok: %d threads, %d jobs claimed once each, %ld locked sections, blobs intact, %d long-poll "
         "claims\n", T, N, sections.load(), N2);
  return 0;
}
