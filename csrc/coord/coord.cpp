// coord.cpp — the framework's control plane: a small multi-threaded TCP
// coordinator that replaces MongoDB in the reference design.
//
// Reference mapping (/root/reference/mapreduce):
//   <db>.task singleton            task.lua:96-193           -> TASK_* ops
//   <db>.map_jobs / red_jobs       task.lua:258-343,job.lua  -> JOB_* ops
//        (claim is ONE atomic op here; the reference did update-then-find,
//         task.lua:294-309, which races — SURVEY.md §5.2)
//   server-side JS mapReduce stats server.lua:155-183        -> JOB_STATS
//   BROKEN -> FAILED sweep         server.lua:189-205        -> JOB_FAIL_BROKEN
//   <db>.errors                    cnn.lua:55-70             -> ERR_* ops
//   GridFS blob store              cnn.lua:41-49, fs.lua     -> BLOB_* ops
//   persistent_table (findAndModify, timestamp CAS, spin lock)
//                                  persistent_table.lua      -> PT_* ops
//   new: job leases (heartbeat + expiry) for dead-worker detection, which the
//   reference lacks, and an append-only journal replayed at
//   start-up for server restart/resume.
//
// Wire format (little endian): request = u32 body_len | u16 op | fields,
// response = u32 body_len | i32 status | fields; field = u32 len | bytes.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

enum Op : uint16_t {
  PING = 1,
  TASK_GET = 10, TASK_SET = 11, TASK_DROP = 12,
  JOB_INSERT = 20, JOB_REMOVE_STATUS = 21, JOB_FAIL_BROKEN = 22, JOB_COUNT = 23, JOB_CLAIM = 24,
  JOB_UPDATE = 25, JOB_GET = 26, JOB_LIST = 27, JOB_DROP = 28, JOB_STATS = 29, JOB_EXPIRE = 30,
  // long polls: JOB_CLAIM_WAIT = wait_ms + JOB_CLAIM's args, blocks (up to
  // wait_ms) until a job can be claimed or the task document changes;
  // WAIT_CHANGE since, wait_ms -> the database's mutation count once it
  // differs from `since` (or at the timeout)
  JOB_CLAIM_WAIT = 31, WAIT_CHANGE = 32,
  ERR_INSERT = 40, ERR_TAKE = 41,
  BLOB_PUT = 50, BLOB_GET = 51, BLOB_LIST = 52, BLOB_DEL = 53,
  // batched forms (one round trip for all outputs of a job, all inputs of a
  // reduce job): PUT_MANY name,data,name,data...; GET_MANY names -> (found, data)...;
  // DEL_MANY names -> count
  BLOB_PUT_MANY = 54, BLOB_GET_MANY = 55, BLOB_DEL_MANY = 56,
  PT_OPEN = 60, PT_UPDATE = 61, PT_LOCK = 62, PT_UNLOCK = 63, PT_DROP = 64,
  DB_DROP = 70, COLLECTIONS = 71, SHUTDOWN = 99,
};

enum Status : int { WAITING = 0, RUNNING = 1, BROKEN = 2, FINISHED = 3, WRITTEN = 4, FAILED = 5 };

bool is_mutating(uint16_t op) {
  switch (op) {
    case TASK_SET: case TASK_DROP: case JOB_INSERT: case JOB_REMOVE_STATUS: case JOB_FAIL_BROKEN:
    case JOB_CLAIM: case JOB_CLAIM_WAIT: case JOB_UPDATE: case JOB_DROP: case JOB_EXPIRE: case ERR_INSERT:
    case ERR_TAKE:
    case BLOB_PUT: case BLOB_DEL: case BLOB_PUT_MANY: case BLOB_DEL_MANY: case PT_OPEN: case PT_UPDATE: case PT_LOCK: case PT_UNLOCK: case PT_DROP:
    case DB_DROP:
      return true;
    default:
      return false;
  }
}

struct Job {
  std::string id, value, worker = "<unknown>", tmpname = "<NONE>";
  int status = WAITING, repetitions = 0;
  double creation_time = 0, started_time = 0, finished_time = 0, written_time = 0, broken_time = 0;
  double cpu_time = 0, real_time = 0, heartbeat = 0;
  bool has_started = false, has_written = false;
  uint64_t seq = 0;
};

struct Collection {
  std::map<uint64_t, std::string> order;            // seq -> id (insertion order = "first match")
  std::unordered_map<std::string, Job> jobs;
  uint64_t next_seq = 1;
};

struct PTable {
  std::string content = "{}";
  int64_t timestamp = 0;
  bool locked = false;
};

struct Db {
  std::map<std::string, std::string> task;  // field -> JSON-encoded value
  bool has_task = false;
  std::map<std::string, Collection> colls;
  std::vector<std::pair<std::string, std::string>> errors;
  // blob bodies are shared and immutable: a read references them (the reply
  // is written after the store lock is released) and a write builds them
  // before taking it, so large blobs are never copied under the lock
  std::map<std::string, std::shared_ptr<const std::string>> blobs;
  std::map<std::string, PTable> ptables;  // key: doc + "\x1f" + name
};

struct Reader {
  const char* p;
  const char* end;
  bool ok = true;
  std::string str() {
    if (end - p < 4) { ok = false; return {}; }
    uint32_t n;
    memcpy(&n, p, 4);
    p += 4;
    if ((size_t)(end - p) < n) { ok = false; return {}; }
    std::string s(p, n);
    p += n;
    return s;
  }
  bool more() const { return p < end; }
};

struct Writer {
  std::string buf;
  // blob bodies referenced by the reply: (offset in buf where the body goes, body)
  std::vector<std::pair<size_t, std::shared_ptr<const std::string>>> refs;
  void blob(std::shared_ptr<const std::string> p) {
    uint32_t n = (uint32_t)p->size();
    buf.append((const char*)&n, 4);
    refs.emplace_back(buf.size(), std::move(p));
  }
  size_t size() const {
    size_t n = buf.size();
    for (auto& r : refs) n += r.second->size();
    return n;
  }
  void str(const std::string& s) {
    uint32_t n = (uint32_t)s.size();
    buf.append((const char*)&n, 4);
    buf.append(s);
  }
  void num(double d) {
    char tmp[64];
    snprintf(tmp, sizeof tmp, "%.17g", d);
    str(tmp);
  }
  void i(long long v) { str(std::to_string(v)); }
};

double to_d(const std::string& s) { return strtod(s.c_str(), nullptr); }
long long to_ll(const std::string& s) { return strtoll(s.c_str(), nullptr, 10); }

void write_job(Writer& w, const Job& j) {
  w.str(j.id); w.str(j.value); w.str(j.worker); w.str(j.tmpname);
  w.i(j.status); w.i(j.repetitions);
  w.num(j.creation_time); w.num(j.has_started ? j.started_time : -1); w.num(j.finished_time);
  w.num(j.has_written ? j.written_time : -1); w.num(j.broken_time); w.num(j.cpu_time); w.num(j.real_time);
  w.num(j.heartbeat);
}

class Store {
 public:
  std::mutex mu;
  std::map<std::string, Db> dbs;
  FILE* journal = nullptr;
  bool replaying = false;
  std::condition_variable cv;
  std::map<std::string, uint64_t> ver;   // per database: mutations so far
  std::map<std::string, uint64_t> tver;  // per database: task-document changes
  bool unchanged = false;  // set by a mutating op that found nothing to change (wakes no long poll)

  // Executes one request; returns status (0 ok, 1 "not found / false", <0 error).
  int exec(uint16_t op, Reader& r, Writer& w) {
    std::string dbname = r.str();
    Db& db = dbs[dbname];
    switch (op) {
      case PING: w.str("pong"); return 0;
      case TASK_GET: {
        // the database's mutation count rides along as field "_ver" (also
        // when there is no task): a long poll from that count waits for
        // whatever changes after this read
        w.str("_ver");
        w.i((long long)ver[dbname]);
        if (!db.has_task) return 1;
        for (auto& kv : db.task) { w.str(kv.first); w.str(kv.second); }
        return 0;
      }
      case TASK_SET: {
        db.has_task = true;
        while (r.more()) { std::string k = r.str(); std::string v = r.str(); if (!r.ok) return -1; db.task[k] = v; }
        return 0;
      }
      case TASK_DROP: db.task.clear(); db.has_task = false; return 0;
      case JOB_INSERT: {
        // one or more (id, value, creation time) triples: a batch is one round trip
        Collection& c = db.colls[r.str()];
        int st = 0;
        do {
          Job j;
          j.id = r.str(); j.value = r.str(); j.creation_time = to_d(r.str());
          if (!r.ok) return -1;
          if (c.jobs.count(j.id)) {  // duplicate key (reference relied on mongo rejection)
            st = 1;
            continue;
          }
          j.seq = c.next_seq++;
          c.order[j.seq] = j.id;
          c.jobs[j.id] = j;
        } while (r.more());
        return st;
      }
      case JOB_REMOVE_STATUS: {
        Collection& c = db.colls[r.str()];
        int mask = (int)to_ll(r.str());
        long long n = 0;
        for (auto it = c.order.begin(); it != c.order.end();) {
          Job& j = c.jobs[it->second];
          if (mask & (1 << j.status)) { c.jobs.erase(it->second); it = c.order.erase(it); ++n; }
          else ++it;
        }
        w.i(n);
        unchanged = n == 0;
        return 0;
      }
      case JOB_FAIL_BROKEN: {
        Collection& c = db.colls[r.str()];
        int maxrep = (int)to_ll(r.str());
        long long n = 0;
        for (auto& kv : c.jobs)
          if (kv.second.status == BROKEN && kv.second.repetitions >= maxrep) { kv.second.status = FAILED; ++n; }
        w.i(n);
        unchanged = n == 0;
        return 0;
      }
      case JOB_COUNT: {
        auto it = db.colls.find(r.str());
        int mask = (int)to_ll(r.str());
        long long n = 0;
        if (it != db.colls.end())
          for (auto& kv : it->second.jobs)
            if (mask == 0 || (mask & (1 << kv.second.status))) ++n;
        w.i(n);
        return 0;
      }
      case JOB_CLAIM_WAIT:
        r.str();  // wait_ms (the waiting is done by handle())
        [[fallthrough]];
      case JOB_CLAIM: {
        // args: coll, worker, tmpname, time, claimable status mask, [ids...]
        Collection& c = db.colls[r.str()];
        std::string worker = r.str(), tmpname = r.str();
        double t = to_d(r.str());
        int mask = (int)to_ll(r.str());
        std::set<std::string> only;
        bool restrict_ids = false;
        while (r.more()) { only.insert(r.str()); restrict_ids = true; }
        if (!r.ok) return -1;
        for (auto& kv : c.order) {
          Job& j = c.jobs[kv.second];
          if (!(mask & (1 << j.status))) continue;
          if (restrict_ids && !only.count(j.id)) continue;
          j.status = RUNNING; j.worker = worker; j.tmpname = tmpname; j.started_time = t; j.has_started = true;
          j.heartbeat = t;
          write_job(w, j);
          return 0;
        }
        return 1;
      }
      case JOB_UPDATE: {
        // args: coll, id, [if_tmpname], then k/v pairs
        Collection& c = db.colls[r.str()];
        std::string id = r.str();
        std::string guard = r.str();
        auto it = c.jobs.find(id);
        if (it == c.jobs.end()) return 1;
        Job& j = it->second;
        if (!guard.empty() && j.tmpname != guard) return 1;  // job was re-assigned: stale writer
        while (r.more()) {
          std::string k = r.str(), v = r.str();
          if (!r.ok) return -1;
          if (k == "status") j.status = (int)to_ll(v);
          else if (k == "finished_time") j.finished_time = to_d(v);
          else if (k == "written_time") { j.written_time = to_d(v); j.has_written = true; }
          else if (k == "cpu_time") j.cpu_time = to_d(v);
          else if (k == "real_time") j.real_time = to_d(v);
          else if (k == "broken_time") j.broken_time = to_d(v);
          else if (k == "heartbeat") j.heartbeat = to_d(v);
          else if (k == "inc_repetitions") j.repetitions += (int)to_ll(v);
          else if (k == "worker") j.worker = v;
          else if (k == "tmpname") j.tmpname = v;
          else if (k == "value") j.value = v;
        }
        write_job(w, j);
        return 0;
      }
      case JOB_GET: {
        auto ci = db.colls.find(r.str());
        std::string id = r.str();
        if (ci == db.colls.end()) return 1;
        auto it = ci->second.jobs.find(id);
        if (it == ci->second.jobs.end()) return 1;
        write_job(w, it->second);
        return 0;
      }
      case JOB_LIST: {
        auto ci = db.colls.find(r.str());
        if (ci == db.colls.end()) return 0;
        for (auto& kv : ci->second.order) write_job(w, ci->second.jobs[kv.second]);
        return 0;
      }
      case JOB_DROP: db.colls.erase(r.str()); return 0;
      case JOB_STATS: {
        auto ci = db.colls.find(r.str());
        double sum_cpu = 0, sum_real = 0, tmin = 0, tmax = 0;
        long long counts[6] = {0, 0, 0, 0, 0, 0};
        bool first = true;
        if (ci != db.colls.end())
          for (auto& kv : ci->second.jobs) {
            const Job& j = kv.second;
            sum_cpu += j.cpu_time;
            sum_real += j.real_time;
            double a = j.has_started ? j.started_time : j.creation_time;
            double b = j.has_written ? j.written_time : j.creation_time;
            if (first || a < tmin) tmin = a;
            if (first || b > tmax) tmax = b;
            first = false;
            if (j.status >= 0 && j.status < 6) counts[j.status]++;
          }
        w.num(sum_cpu); w.num(sum_real); w.num(tmax - tmin);
        for (int k = 0; k < 6; ++k) w.i(counts[k]);
        return 0;
      }
      case JOB_EXPIRE: {
        Collection& c = db.colls[r.str()];
        double now = to_d(r.str()), lease = to_d(r.str());
        long long n = 0;
        for (auto& kv : c.jobs) {
          Job& j = kv.second;
          if (j.status == RUNNING && j.heartbeat < now - lease) {
            j.status = BROKEN; j.repetitions += 1; j.broken_time = now; ++n;
          }
        }
        w.i(n);
        unchanged = n == 0;
        return 0;
      }
      case ERR_INSERT: {
        std::string who = r.str(), msg = r.str();
        db.errors.emplace_back(who, msg);
        return 0;
      }
      case ERR_TAKE: {
        unchanged = db.errors.empty();
        for (auto& e : db.errors) { w.str(e.first); w.str(e.second); }
        db.errors.clear();
        return 0;
      }
      case BLOB_PUT: {
        std::string n = r.str();
        db.blobs[n] = std::make_shared<const std::string>(r.str());
        return r.ok ? 0 : -1;
      }
      case BLOB_GET: {
        auto it = db.blobs.find(r.str());
        if (it == db.blobs.end()) return 1;
        w.blob(it->second);
        return 0;
      }
      case BLOB_LIST: {
        std::string prefix = r.str();
        for (auto it = db.blobs.lower_bound(prefix); it != db.blobs.end(); ++it) {
          if (it->first.compare(0, prefix.size(), prefix) != 0) break;
          w.str(it->first);
          w.i((long long)it->second->size());
        }
        return 0;
      }
      case BLOB_DEL: { w.i((long long)db.blobs.erase(r.str())); return 0; }
      case BLOB_PUT_MANY: {
        while (r.more() && r.ok) {
          std::string n = r.str();
          std::string d = r.str();
          if (!r.ok) return -1;
          db.blobs[n] = std::make_shared<const std::string>(std::move(d));
        }
        return r.ok ? 0 : -1;
      }
      case BLOB_GET_MANY: {
        while (r.more() && r.ok) {
          auto it = db.blobs.find(r.str());
          if (it == db.blobs.end()) {
            w.i(0);
            w.str(std::string());
          } else {
            w.i(1);
            w.blob(it->second);
          }
        }
        return r.ok ? 0 : -1;
      }
      case BLOB_DEL_MANY: {
        long long c = 0;
        while (r.more() && r.ok) c += (long long)db.blobs.erase(r.str());
        w.i(c);
        return 0;
      }
      case PT_OPEN: {
        std::string d_ = r.str(); std::string key = d_ + "\x1f" + r.str();
        PTable& t = db.ptables[key];
        w.str(t.content); w.i(t.timestamp); w.i(t.locked ? 1 : 0);
        return 0;
      }
      case PT_UPDATE: {
        // args: doc, name, dirty(0/1), expected_ts, content
        std::string d_ = r.str(); std::string key = d_ + "\x1f" + r.str();
        bool dirty = to_ll(r.str()) != 0;
        long long expect = to_ll(r.str());
        std::string content = r.str();
        PTable& t = db.ptables[key];
        int st = 0;
        if (dirty) {
          if (t.timestamp == expect) { t.content = content; t.timestamp += 1; }
          else st = 1;  // inconsistent: someone else updated first
        }
        w.str(t.content); w.i(t.timestamp); w.i(t.locked ? 1 : 0);
        return st;
      }
      case PT_LOCK: {
        std::string d_ = r.str(); std::string key = d_ + "\x1f" + r.str();
        PTable& t = db.ptables[key];
        bool was = t.locked;
        t.locked = true;
        w.i(was ? 1 : 0);
        return 0;
      }
      case PT_UNLOCK: {
        std::string d_ = r.str(); std::string key = d_ + "\x1f" + r.str();
        PTable& t = db.ptables[key];
        bool was = t.locked;
        t.locked = false;
        w.i(was ? 1 : 0);
        return 0;
      }
      case PT_DROP: {
        std::string d_ = r.str(); std::string key = d_ + "\x1f" + r.str();
        PTable& t = db.ptables[key];
        t.content = "{}";
        t.timestamp += 1;
        t.locked = false;
        w.str(t.content); w.i(t.timestamp); w.i(0);
        return 0;
      }
      case DB_DROP: dbs.erase(dbname); return 0;
      case COLLECTIONS: {
        for (auto& kv : db.colls) w.str(kv.first);
        return 0;
      }
      default: return -2;
    }
  }

  // Journal record: u32 length | u32 FNV-1a of the body | body.  A record cut
  // short by a crash (or one whose checksum does not match) ends the replay,
  // and the file is truncated there before appending resumes, so the next
  // record never lands behind a stale length prefix.
  static uint32_t body_sum(const std::string& body) {
    uint32_t h = 2166136261u;
    for (unsigned char c : body) h = (h ^ c) * 16777619u;
    return h;
  }

  void log(const std::string& body) {
    if (!journal || replaying) return;
    uint32_t hdr[2] = {(uint32_t)body.size(), body_sum(body)};
    fwrite(hdr, 4, 2, journal);
    fwrite(body.data(), 1, body.size(), journal);
    fflush(journal);
  }

  // (Deadlines are on system_clock: a condition-variable wait on it is a
  // pthread_cond_timedwait, which ThreadSanitizer understands; steady_clock
  // waits go through pthread_cond_clockwait, which it does not intercept.)
  // Long polls: every mutation of a database bumps its count and wakes the
  // waiters (one condition variable for the store; waits are short and few:
  // one per idle worker and one for the server's monitor).

  static std::string db_of(const std::string& body) {
    Reader r{body.data() + 2, body.data() + body.size()};
    return r.str();
  }

  // A claim that found nothing: wait for a mutation of the database and claim
  // again, until the deadline; a change of the task document ends the wait
  // (the worker re-reads the task: the phase may have changed).
  int claim_wait(const std::string& body, Writer& w, std::unique_lock<std::mutex>& g) {
    Reader r{body.data() + 2, body.data() + body.size()};
    const std::string db = r.str();
    const double ms = to_d(r.str());
    if (!r.ok || !(ms > 0)) return 1;
    const auto deadline = std::chrono::system_clock::now() + std::chrono::microseconds((long long)(ms * 1000.0));
    const uint64_t tv = tver[db];
    uint64_t v = ver[db];
    for (;;) {
      if (!cv.wait_until(g, deadline, [&] { return ver[db] != v; })) return 1;
      if (tver[db] != tv) return 1;
      v = ver[db];
      Reader r2{body.data() + 2, body.data() + body.size()};
      Writer w2;
      const int st = exec(JOB_CLAIM_WAIT, r2, w2);
      if (st != 1) {
        w = std::move(w2);
        return st;
      }
    }
  }

  int wait_change(Reader& r, Writer& w, std::unique_lock<std::mutex>& g) {
    const std::string db = r.str();
    const uint64_t since = (uint64_t)to_ll(r.str());
    const double ms = to_d(r.str());
    if (!r.ok) return -1;
    if (ms > 0)
      cv.wait_until(g, std::chrono::system_clock::now() + std::chrono::microseconds((long long)(ms * 1000.0)),
                    [&] { return ver[db] != since; });
    w.i((long long)ver[db]);
    return 0;
  }

  // BLOB_PUT / BLOB_PUT_MANY with the bodies built before the lock is taken
  int put_blobs(uint16_t op, const std::string& body, Writer& w) {
    Reader r{body.data() + 2, body.data() + body.size()};
    const std::string dbname = r.str();
    std::vector<std::pair<std::string, std::shared_ptr<const std::string>>> items;
    do {
      std::string n = r.str();
      std::string d = r.str();
      if (!r.ok) return -1;
      items.emplace_back(std::move(n), std::make_shared<const std::string>(std::move(d)));
    } while (op == BLOB_PUT_MANY && r.more());
    std::unique_lock<std::mutex> g(mu);
    Db& db = dbs[dbname];
    for (auto& it : items) db.blobs[it.first] = std::move(it.second);
    log(body);
    ++ver[dbname];
    cv.notify_all();
    (void)w;
    return 0;
  }

  int handle(const std::string& body, Writer& w) {
    if (body.size() < 2) return -1;
    uint16_t op;
    memcpy(&op, body.data(), 2);
    if ((op == BLOB_PUT || op == BLOB_PUT_MANY) && !replaying) return put_blobs(op, body, w);
    Reader r{body.data() + 2, body.data() + body.size()};
    std::unique_lock<std::mutex> g(mu);
    if (op == WAIT_CHANGE) return replaying ? 0 : wait_change(r, w, g);
    unchanged = false;
    int st = exec(op, r, w);
    if (!r.ok) return -1;
    if (op == JOB_CLAIM_WAIT && st == 1 && !replaying) st = claim_wait(body, w, g);
    if (is_mutating(op) && st >= 0) log(body);
    if (is_mutating(op) && st == 0 && !unchanged) {  // (a claim that found nothing wakes nobody)
      const std::string db = db_of(body);
      ++ver[db];
      if (op == TASK_SET || op == TASK_DROP || op == DB_DROP) ++tver[db];
      cv.notify_all();
    }
    return st;
  }

  // Journal file: an 8-byte magic/version header, then records
  // len | FNV-1a(body) | body.  Replay stops at the first record that is short
  // (a write torn by a crash: the tail is cut there) or whose checksum does
  // not match; such a tail is kept as <path>.corrupt before the journal is
  // cut back to the last intact record.  A length field larger than the bytes
  // left is a torn tail (no allocation is made from it).  A file without the
  // header whose first record is intact is a journal of the previous build
  // (the same records, no header): it is replayed and rewritten with the
  // header (in place, through a temporary file and a rename).  Any other
  // file is refused (never truncated: it may be another program's).
  static constexpr char JMAGIC[8] = {'M', 'R', 'J', 'N', 'L', 0, 0, 2};

  // Replays the records from the current position; returns the end of the
  // last intact record.
  long replay_records(FILE* f, long size, bool& corrupt) {
    long good = ftell(f);
    corrupt = false;
    replaying = true;
    for (;;) {
      uint32_t hdr[2];
      const long at = ftell(f);
      if (at == size) break;
      if (fread(hdr, 4, 2, f) != 2) break;                 // torn header
      if ((long)hdr[0] > size - at - 8) break;             // torn body (or a garbled length)
      std::string body(hdr[0], '\0');
      if (fread(&body[0], 1, hdr[0], f) != hdr[0]) break;
      if (body_sum(body) != hdr[1]) {
        corrupt = true;
        break;
      }
      Writer w;
      handle(body, w);
      good = ftell(f);
    }
    replaying = false;
    return good;
  }

  // The first record of a headerless file is intact (a legacy journal).
  static bool legacy_journal(FILE* f, long size) {
    uint32_t hdr[2];
    fseek(f, 0, SEEK_SET);
    if (size < 8 || fread(hdr, 4, 2, f) != 2 || (long)hdr[0] > size - 8) return false;
    std::string body(hdr[0], '\0');
    if (hdr[0] && fread(&body[0], 1, hdr[0], f) != hdr[0]) return false;
    fseek(f, 0, SEEK_SET);
    return body_sum(body) == hdr[1];
  }

  static void keep_tail(FILE* f, const char* path, long good, long size, bool corrupt) {
    std::string keep = std::string(path) + ".corrupt";
    FILE* c = fopen(keep.c_str(), "wb");
    if (c) {
      fseek(f, good, SEEK_SET);
      char buf[65536];
      size_t k;
      while ((k = fread(buf, 1, sizeof buf, f)) > 0) fwrite(buf, 1, k, c);
      fclose(c);
    }
    fprintf(stderr, "coordinator: journal %s: %s at byte %ld of %ld, replayed the intact prefix (tail kept in %s)\n",
            path, corrupt ? "checksum mismatch" : "torn record", good, size, keep.c_str());
  }

  bool open_journal(const char* path) {
    if (!path || !*path) return true;
    FILE* f = fopen(path, "rb");
    long size = 0;
    if (f) {
      fseek(f, 0, SEEK_END);
      size = ftell(f);
      fseek(f, 0, SEEK_SET);
    }
    if (f && size > 0) {
      char magic[8];
      bool corrupt = false;
      if (fread(magic, 1, 8, f) != 8 || memcmp(magic, JMAGIC, 8) != 0) {
        if (!legacy_journal(f, size)) {
          fclose(f);
          fprintf(stderr, "coordinator: %s is not a journal of this format (header mismatch); refusing to use it\n",
                  path);
          return false;
        }
        // a journal of the previous build: replay it, then rewrite it with
        // the header (the old file is replaced only once the new one is whole)
        const long good = replay_records(f, size, corrupt);
        if (good < size) keep_tail(f, path, good, size, corrupt);
        std::string tmp = std::string(path) + ".upgrade";
        FILE* n = fopen(tmp.c_str(), "wb");
        if (!n) {
          fclose(f);
          return false;
        }
        fwrite(JMAGIC, 1, 8, n);
        fseek(f, 0, SEEK_SET);
        char buf[65536];
        long left = good;
        while (left > 0) {
          size_t k = fread(buf, 1, (size_t)(left < (long)sizeof buf ? left : (long)sizeof buf), f);
          if (k == 0) break;
          fwrite(buf, 1, k, n);
          left -= (long)k;
        }
        fclose(f);
        // durable before it replaces the only copy of the state: the new file
        // synced, the old one kept as <path>.legacy (a hard link) until the
        // upgraded journal has been reopened, the directory entry synced
        // (a power loss right after the rename could otherwise
        // leave an empty journal, read as a fresh one)
        const bool synced = fflush(n) == 0 && fsync(fileno(n)) == 0;
        if (fclose(n) != 0 || !synced || left != 0) return false;
        legacy = std::string(path) + ".legacy";
        unlink(legacy.c_str());
        if (link(path, legacy.c_str()) != 0) legacy.clear();
        if (rename(tmp.c_str(), path) != 0) return false;
        sync_dir(path);
        fprintf(stderr, "coordinator: journal %s upgraded from the headerless format (%ld bytes replayed)\n", path,
                good);
      } else {
        const long good = replay_records(f, size, corrupt);
        if (good < size) keep_tail(f, path, good, size, corrupt);
        fclose(f);
        if (truncate(path, good) != 0) return false;
      }
    } else {
      if (f) fclose(f);
      FILE* n = fopen(path, "wb");
      if (!n) return false;
      fwrite(JMAGIC, 1, 8, n);
      fclose(n);
    }
    journal = fopen(path, "ab");
    if (journal != nullptr && !legacy.empty()) {
      unlink(legacy.c_str());  // the upgraded journal is in use: the old copy can go
      legacy.clear();
    }
    return journal != nullptr;
  }

  std::string legacy;  // the pre-upgrade journal, kept until the upgraded one is reopened

  static void sync_dir(const char* path) {
    std::string d(path);
    const size_t k = d.find_last_of('/');
    d = k == std::string::npos ? std::string(".") : (k == 0 ? std::string("/") : d.substr(0, k));
    const int fd = ::open(d.c_str(), O_RDONLY | O_DIRECTORY);
    if (fd >= 0) {
      fsync(fd);
      ::close(fd);
    }
  }
};

bool read_full(int fd, void* buf, size_t n) {
  char* p = (char*)buf;
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool write_full(int fd, const void* buf, size_t n) {
  const char* p = (const char*)buf;
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

struct Server {
  Store store;
  int listen_fd = -1;
  int port = 0;
  std::atomic<bool> stop{false};
  std::thread acceptor;
  std::mutex conn_mu;
  std::vector<std::thread> conns;

  void serve_conn(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    for (;;) {
      uint32_t n;
      if (!read_full(fd, &n, 4)) break;
      std::string body(n, '\0');
      if (n && !read_full(fd, &body[0], n)) break;
      uint16_t op = 0;
      if (n >= 2) memcpy(&op, body.data(), 2);
      Writer w;
      int st = store.handle(body, w);
      uint32_t rn = (uint32_t)(4 + w.size());
      std::string out;
      out.append((const char*)&rn, 4);
      out.append((const char*)&st, 4);
      bool ok = true;
      if (w.refs.empty()) {
        out.append(w.buf);
        ok = write_full(fd, out.data(), out.size());
      } else {  // referenced blob bodies go straight from the store (no copy, no lock)
        size_t at = 0;
        for (auto& ref : w.refs) {
          out.append(w.buf, at, ref.first - at);
          at = ref.first;
          if (!(ok = write_full(fd, out.data(), out.size()))) break;
          out.clear();
          if (!(ok = write_full(fd, ref.second->data(), ref.second->size()))) break;
        }
        if (ok) {
          out.append(w.buf, at, std::string::npos);
          ok = write_full(fd, out.data(), out.size());
        }
      }
      if (!ok) break;
      if (op == SHUTDOWN) { stop = true; ::shutdown(listen_fd, SHUT_RDWR); break; }
    }
    ::close(fd);
  }

  int start(const char* host, int want_port, const char* journal) {
    if (!store.open_journal(journal)) return -1;
    listen_fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (listen_fd < 0) return -1;
    int one = 1;
    setsockopt(listen_fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)want_port);
    a.sin_addr.s_addr = (host && *host) ? inet_addr(host) : htonl(INADDR_ANY);
    if (::bind(listen_fd, (sockaddr*)&a, sizeof a) < 0) return -1;
    if (::listen(listen_fd, 256) < 0) return -1;
    socklen_t len = sizeof a;
    getsockname(listen_fd, (sockaddr*)&a, &len);
    port = ntohs(a.sin_port);
    acceptor = std::thread([this] {
      while (!stop) {
        int fd = ::accept(listen_fd, nullptr, nullptr);
        if (fd < 0) {
          if (stop) break;
          if (errno == EINTR || errno == ECONNABORTED) continue;
          break;
        }
        std::lock_guard<std::mutex> g(conn_mu);
        conns.emplace_back([this, fd] { serve_conn(fd); });
        conns.back().detach();
      }
    });
    return port;
  }
};

std::mutex g_mu;
// Leaked on purpose: detached server threads may outlive static destruction.
std::vector<Server*>* g_servers = new std::vector<Server*>();

}  // namespace

extern "C" {

// Start a coordinator in a background thread of this process.  Returns the
// bound port (>0) or -1.  `journal` (may be NULL/"") enables durability: every
// mutating request is appended and replayed on the next start.
int mrc_start(const char* host, int port, const char* journal) {
  Server* s = new Server();
  int p = s->start(host, port, journal);
  if (p <= 0) {
    delete s;
    return -1;
  }
  s->acceptor.detach();
  std::lock_guard<std::mutex> g(g_mu);
  g_servers->push_back(s);
  return p;
}

// Run a coordinator in the calling thread until a SHUTDOWN request arrives.
int mrc_serve_forever(const char* host, int port, const char* journal) {
  int p = mrc_start(host, port, journal);
  if (p <= 0) return -1;
  fprintf(stderr, "# coordinator listening on port %d\n", p);
  fflush(stderr);
  Server* s;
  {
    std::lock_guard<std::mutex> g(g_mu);
    s = g_servers->back();
  }
  while (!s->stop) std::this_thread::sleep_for(std::chrono::milliseconds(50));
  return 0;
}

}  // extern "C"
