// Bulk row writer: one SQLite write transaction driven by its own thread.
//
// The indexer replaces a project's class / method / parameter rows in one
// transaction (pipeline Phase 1).  Through Python's sqlite3 module every row
// costs a GIL round-trip, so the B-tree work can neither leave the
// interpreter nor overlap the Python code that builds the rows and the graph
// JSON.  A BulkWriter opens its own connection on a worker thread, runs the
// setup statements (the old rows' deletes) as soon as it is created, then
// inserts each queued batch; the producer only pays for copying the values
// out of Python objects.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <chrono>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace dbw {

// Text values are views: the caller keeps the bytes alive until wait()
// returns (the Python wrapper holds the row tuples, whose str objects own
// their UTF-8 buffers) -- no per-value copy on the producer side.
struct Value {
    enum Kind : uint8_t { Null, Int, Real, Text } kind = Null;
    int32_t n = 0;
    union {
        int64_t i;
        double d;
        const char* p;
    };
    Value() : i(0) {}
};

// rows flattened row-major: values.size() == ncols * rows.  Text values
// that no caller-owned object holds live in ``owned`` (a deque: element
// addresses stay put as it grows).
struct Batch {
    std::string sql;
    int ncols = 0;
    std::vector<Value> values;
    std::deque<std::string> owned;
    std::shared_ptr<const void> keep;  // whatever else the text values view (released after the insert)
};

class BulkWriter {
  public:
    // `setup`: statements run right after BEGIN IMMEDIATE, in order.
    BulkWriter(std::string path, int busy_timeout_ms, std::vector<Batch> setup);
    ~BulkWriter();
    BulkWriter(const BulkWriter&) = delete;
    BulkWriter& operator=(const BulkWriter&) = delete;

    void put(Batch batch);
    void commit();             // no more batches: COMMIT once the queue drains
    void abort();              // ROLLBACK (queued batches are dropped) and join
    std::string wait();        // join; "" on success, else the error message
    int64_t rows_written() const { return rows_written_; }
    // wall time of the writer thread's phases (valid after wait()): the
    // setup statements (old rows' deletes), the inserts, the COMMIT
    double setup_ms() const { return setup_ms_; }
    double rows_ms() const { return rows_ms_; }
    double commit_ms() const { return commit_ms_; }
    double idle_ms() const { return idle_ms_; }  // waits for rows between the setup and the commit request
    double free_ms() const { return free_ms_; }  // releasing inserted batches (handing them to the reaper)
    double open_ms() const { return open_ms_; }  // from construction to BEGIN (thread start, open, pragmas)
    // steady_clock (CLOCK_MONOTONIC, Python's time.perf_counter on Linux) seconds of the writer's milestones
    static double secs(std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double>(t.time_since_epoch()).count();
    }
    double t_start() const { return secs(t_start_); }
    double t_setup() const { return secs(t_setup_); }
    double t_commit() const { return secs(t_commit_); }
    double t_end() const { return secs(t_end_); }

  private:
    enum class Op { Rows, Commit, Abort };
    struct Item {
        Op op;
        Batch batch;
    };
    void run();
    void push(Item it);
    bool pop(Item& out);

    std::string path_;
    int busy_ms_;
    std::vector<Batch> setup_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Item> queue_;
    std::thread thread_;
    std::string error_;
    int64_t rows_written_ = 0;
    double setup_ms_ = 0, rows_ms_ = 0, commit_ms_ = 0, idle_ms_ = 0, open_ms_ = 0, free_ms_ = 0;
    std::chrono::steady_clock::time_point t_start_ = std::chrono::steady_clock::now();
    std::chrono::steady_clock::time_point t_setup_{}, t_commit_{}, t_end_{};
    bool joined_ = false;
    bool commit_requested_ = false;
};

}  // namespace dbw
