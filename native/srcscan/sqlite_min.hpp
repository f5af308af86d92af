// The handful of SQLite C API entry points the bulk writer uses, declared
// against the stable public ABI of the system libsqlite3.so.0 (the library the
// Python sqlite3 module itself links).  The image ships the runtime library
// without its development header, so the prototypes live here.
#pragma once

#include <cstdint>

extern "C" {
struct sqlite3;
struct sqlite3_stmt;
typedef int64_t sqlite3_int64;

int sqlite3_open_v2(const char* filename, sqlite3** db, int flags, const char* vfs);
int sqlite3_close_v2(sqlite3* db);
int sqlite3_busy_timeout(sqlite3* db, int ms);
int sqlite3_exec(sqlite3* db, const char* sql, int (*cb)(void*, int, char**, char**), void* arg, char** errmsg);
void sqlite3_free(void* p);
int sqlite3_prepare_v2(sqlite3* db, const char* sql, int n, sqlite3_stmt** stmt, const char** tail);
int sqlite3_bind_null(sqlite3_stmt* s, int i);
int sqlite3_bind_int64(sqlite3_stmt* s, int i, sqlite3_int64 v);
int sqlite3_bind_double(sqlite3_stmt* s, int i, double v);
int sqlite3_bind_text(sqlite3_stmt* s, int i, const char* v, int n, void (*destructor)(void*));
int sqlite3_bind_parameter_count(sqlite3_stmt* s);
int sqlite3_step(sqlite3_stmt* s);
int sqlite3_reset(sqlite3_stmt* s);
int sqlite3_finalize(sqlite3_stmt* s);
const char* sqlite3_errmsg(sqlite3* db);
}

namespace sqlite_min {
constexpr int OK = 0;
constexpr int ROW = 100;
constexpr int DONE = 101;
constexpr int OPEN_READWRITE = 0x00000002;
constexpr int OPEN_NOMUTEX = 0x00008000;
inline void (*const STATIC)(void*) = nullptr;  // bound buffers outlive the step
}  // namespace sqlite_min
