#include "bulkwriter.hpp"

#include <cstdlib>

#include <chrono>
#include <stdexcept>

#include "sqlite_min.hpp"

namespace dbw {

namespace {

// Inserted batches are released here, off the writer thread: freeing an
// analysis' ~13k rows (their value arrays, owned text and the scan result
// they view) took 3-4 ms of the writer's critical path on the MI355X host
// (large blocks go back to the kernel one munmap at a time).  One process-
// lifetime thread; batches hold no Python objects.
class Reaper {
  public:
    static void give(std::vector<Batch>&& dead) {
        if (dead.empty()) return;
        static Reaper* r = new Reaper();  // never destroyed: its thread may outlive static teardown
        {
            std::lock_guard<std::mutex> g(r->mu_);
            r->queue_.push_back(std::move(dead));
        }
        r->cv_.notify_one();
    }

  private:
    Reaper() { std::thread([this] { loop(); }).detach(); }
    void loop() {
        for (;;) {
            std::vector<Batch> dead;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return !queue_.empty(); });
                dead = std::move(queue_.front());
                queue_.pop_front();
            }
        }  // `dead` released here
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::vector<Batch>> queue_;
};

struct Conn {
    sqlite3* db = nullptr;
    ~Conn() {
        if (db) sqlite3_close_v2(db);
    }
    void exec(const char* sql) {
        char* err = nullptr;
        if (sqlite3_exec(db, sql, nullptr, nullptr, &err) != sqlite_min::OK) {
            std::string m = err ? err : sqlite3_errmsg(db);
            sqlite3_free(err);
            throw std::runtime_error(std::string(sql) + ": " + m);
        }
    }
    int64_t run(const Batch& b) {
        sqlite3_stmt* st = nullptr;
        if (sqlite3_prepare_v2(db, b.sql.c_str(), static_cast<int>(b.sql.size()), &st, nullptr) != sqlite_min::OK)
            throw std::runtime_error("prepare: " + b.sql + ": " + sqlite3_errmsg(db));
        struct Fin {
            sqlite3_stmt* s;
            ~Fin() { sqlite3_finalize(s); }
        } fin{st};
        const int n = b.ncols;
        if (sqlite3_bind_parameter_count(st) != n)
            throw std::runtime_error("parameter count mismatch for: " + b.sql);
        const size_t rows = n ? b.values.size() / n : 1;
        for (size_t r = 0; r < rows; ++r) {
            const Value* v = n ? &b.values[r * n] : nullptr;
            for (int c = 0; c < n; ++c) {
                const Value& x = v[c];
                int rc = sqlite_min::OK;
                switch (x.kind) {
                    case Value::Null: rc = sqlite3_bind_null(st, c + 1); break;
                    case Value::Int: rc = sqlite3_bind_int64(st, c + 1, x.i); break;
                    case Value::Real: rc = sqlite3_bind_double(st, c + 1, x.d); break;
                    case Value::Text:
                        rc = sqlite3_bind_text(st, c + 1, x.p, x.n, sqlite_min::STATIC);
                        break;
                }
                if (rc != sqlite_min::OK) throw std::runtime_error(std::string("bind: ") + sqlite3_errmsg(db));
            }
            int rc = sqlite3_step(st);
            if (rc != sqlite_min::DONE && rc != sqlite_min::ROW)
                throw std::runtime_error("step: " + b.sql + ": " + sqlite3_errmsg(db));
            sqlite3_reset(st);
        }
        return static_cast<int64_t>(rows);
    }
};

}  // namespace

BulkWriter::BulkWriter(std::string path, int busy_timeout_ms, std::vector<Batch> setup)
    : path_(std::move(path)), busy_ms_(busy_timeout_ms), setup_(std::move(setup)) {
    thread_ = std::thread([this] { run(); });
}

BulkWriter::~BulkWriter() {
    if (joined_) return;
    if (commit_requested_)
        wait();
    else
        abort();
}

void BulkWriter::push(Item it) {
    {
        std::lock_guard<std::mutex> g(mu_);
        queue_.push_back(std::move(it));
    }
    cv_.notify_one();
}

bool BulkWriter::pop(Item& out) {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [this] { return !queue_.empty(); });
    out = std::move(queue_.front());
    queue_.pop_front();
    return true;
}

void BulkWriter::put(Batch batch) { push(Item{Op::Rows, std::move(batch)}); }

void BulkWriter::commit() {
    commit_requested_ = true;
    push(Item{Op::Commit, {}});
}

void BulkWriter::abort() {
    {
        std::lock_guard<std::mutex> g(mu_);
        queue_.push_front(Item{Op::Abort, {}});  // ahead of anything still queued
    }
    cv_.notify_one();
    wait();
}

std::string BulkWriter::wait() {
    if (!joined_) {
        if (thread_.joinable()) thread_.join();
        joined_ = true;
    }
    return error_;
}

void BulkWriter::run() {
    Conn c;
    bool in_tx = false;
    try {
        if (sqlite3_open_v2(path_.c_str(), &c.db, sqlite_min::OPEN_READWRITE | sqlite_min::OPEN_NOMUTEX, nullptr) !=
            sqlite_min::OK)
            throw std::runtime_error("open " + path_ + ": " + (c.db ? sqlite3_errmsg(c.db) : "out of memory"));
        sqlite3_busy_timeout(c.db, busy_ms_);
        // the same per-connection settings as the Python connections, minus
        // foreign-key enforcement: parents are inserted before children and
        // children deleted before parents by construction
        c.exec("PRAGMA synchronous = NORMAL");
        c.exec("PRAGMA temp_store = MEMORY");
        c.exec("PRAGMA cache_size = -65536");
        c.exec("PRAGMA foreign_keys = OFF");
        {
            // each analysis opens a fresh connection, so its page cache starts
            // cold: the old rows' deletes read their B-tree pages through the
            // memory map instead of one read() per page
            static const long long mmap_bytes = [] {
                const char* e = std::getenv("DMCP_WRITER_MMAP");
                return e ? std::atoll(e) : (1LL << 30);
            }();
            if (mmap_bytes > 0) {
                const std::string q = "PRAGMA mmap_size = " + std::to_string(mmap_bytes);
                c.exec(q.c_str());
            }
        }
        using clock = std::chrono::steady_clock;
        auto ms = [](clock::time_point a, clock::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        auto t0 = clock::now();
        open_ms_ = ms(t_start_, t0);
        c.exec("BEGIN IMMEDIATE");
        in_tx = true;
        for (const Batch& b : setup_) c.run(b);
        setup_.clear();
        setup_ms_ = ms(t0, clock::now());
        t_setup_ = clock::now();
        // inserted batches, handed to the reaper in groups as they are
        // inserted: the writer never frees them itself, and an analysis' row
        // buffers (with the scan result they view) are not all held until
        // the COMMIT -- peak writer memory stays a group, not the repository
        constexpr size_t kReapGroup = 16;
        std::vector<Batch> dead;
        dead.reserve(kReapGroup);
        static const bool reap = [] {
            const char* e = std::getenv("DMCP_WRITER_REAPER");
            return e == nullptr || e[0] != '0';
        }();
        for (;;) {
            Item it;
            auto tw = clock::now();
            pop(it);
            idle_ms_ += ms(tw, clock::now());  // waiting for the producer's rows
            if (it.op == Op::Abort) {
                c.exec("ROLLBACK");
                in_tx = false;
                error_ = "aborted";
                return;
            }
            if (it.op == Op::Commit) {
                auto tc = clock::now();
                c.exec("COMMIT");
                commit_ms_ = ms(tc, clock::now());
                t_commit_ = tc;
                t_end_ = clock::now();
                Reaper::give(std::move(dead));
                in_tx = false;
                return;
            }
            auto tr = clock::now();
            rows_written_ += c.run(it.batch);
            auto tf = clock::now();
            rows_ms_ += ms(tr, tf);
            if (reap) {
                dead.push_back(std::move(it.batch));
                if (dead.size() >= kReapGroup) {
                    Reaper::give(std::move(dead));
                    dead = std::vector<Batch>();
                    dead.reserve(kReapGroup);
                }
            } else
                Batch(std::move(it.batch));  // (DMCP_WRITER_REAPER=0: released here, as before)
            free_ms_ += ms(tf, clock::now());
        }
    } catch (const std::exception& e) {
        error_ = e.what();
        if (in_tx && c.db) sqlite3_exec(c.db, "ROLLBACK", nullptr, nullptr, nullptr);
    }
}

}  // namespace dbw
