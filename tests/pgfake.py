"""A PostgreSQL wire-protocol (v3) server for tests, executing on SQLite.

No PostgreSQL server exists on this host; the reference runs its repository
tests on a Testcontainers ``postgres:14``.  This server speaks the real
protocol -- SSLRequest refusal, startup, trust / cleartext / MD5 /
SCRAM-SHA-256 authentication, simple and extended query messages, error
responses with SQLSTATE codes, transaction status in ReadyForQuery, the
"skip until Sync" error rule -- so :mod:`dmcp.store.pgwire` and
:mod:`dmcp.store.pg` are exercised byte for byte.  Statements run on one
SQLite database (``$n`` placeholders -> ``?n``; PostgreSQL-only DDL such as
``CREATE SCHEMA`` / ``SET`` is acknowledged and skipped), so SQL *semantics*
specific to PostgreSQL are not what these tests pin (parity unpinned for a
real server).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import re
import socket
import sqlite3
import struct
import threading
from typing import Dict, List, Optional, Tuple

_DOLLAR = re.compile(r"'(?:[^']|'')*'|\$(\d+)")


def _to_sqlite(sql: str) -> str:
    return _DOLLAR.sub(lambda m: f"?{m.group(1)}" if m.group(1) else m.group(0), sql)


def _param(raw: Optional[bytes]):
    if raw is None:
        return None
    s = raw.decode("utf-8")
    if re.fullmatch(r"-?\d{1,18}", s):
        return int(s)
    return s


def _sqlstate(e: Exception) -> str:
    m = str(e).lower()
    if "unique" in m:
        return "23505"
    if "foreign key" in m:
        return "23503"
    if "not null" in m:
        return "23502"
    if "no such table" in m:
        return "42P01"
    if "syntax" in m:
        return "42601"
    return "XX000"


class FakePgServer:
    """``with FakePgServer(auth="scram", password="pw") as srv: srv.port``."""

    def __init__(self, db_path: str, auth: str = "trust", user: str = "dmcp", password: str = "secret") -> None:
        self.db_path = db_path
        self.auth = auth
        self.user = user
        self.password = password
        self.statements: List[str] = []  # every statement text received (tests inspect it)
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._sock.bind(("127.0.0.1", 0))
        self._sock.listen(64)
        self.port = self._sock.getsockname()[1]
        self._stop = False
        self._threads: List[threading.Thread] = []
        self._acceptor = threading.Thread(target=self._accept, daemon=True)
        self._acceptor.start()

    def __enter__(self) -> "FakePgServer":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def url(self, schema: Optional[str] = "domain_mcp", with_password: bool = True) -> str:
        cred = f"{self.user}:{self.password}@" if with_password else f"{self.user}@"
        return f"postgresql://{cred}127.0.0.1:{self.port}/testdb" + (f"?currentSchema={schema}" if schema else "")

    def close(self) -> None:
        self._stop = True
        try:
            socket.create_connection(("127.0.0.1", self.port), timeout=1).close()
        except OSError:
            pass
        self._sock.close()

    def _accept(self) -> None:
        while not self._stop:
            try:
                conn, _ = self._sock.accept()
            except OSError:
                return
            if self._stop:
                conn.close()
                return
            t = threading.Thread(target=_Session(self, conn).run, daemon=True)
            t.start()
            self._threads.append(t)


class _Session:
    def __init__(self, server: FakePgServer, sock: socket.socket) -> None:
        self.srv = server
        self.sock = sock
        self.buf = b""
        self.db = sqlite3.connect(server.db_path, isolation_level=None, check_same_thread=False, timeout=30)
        self.db.execute("PRAGMA foreign_keys = ON")
        self.db.execute("PRAGMA journal_mode = WAL")
        self.failed = False       # error inside a transaction block
        self.skip = False         # extended protocol: error, discard until Sync
        self.prepared: Dict[str, str] = {}
        self.portal: Optional[Tuple[str, list]] = None
        self.result: Optional[Tuple[list, list, str]] = None

    # ------------------------------------------------------------ transport
    def recv(self, n: int) -> bytes:
        while len(self.buf) < n:
            chunk = self.sock.recv(65536)
            if not chunk:
                raise ConnectionError
            self.buf += chunk
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def send(self, kind: bytes, body: bytes = b"") -> None:
        self.sock.sendall(kind + struct.pack("!i", len(body) + 4) + body)

    def error(self, e: Exception, code: Optional[str] = None) -> None:
        fields = b"SERROR\0VERROR\0C" + (code or _sqlstate(e)).encode() + b"\0M" + str(e).encode() + b"\0\0"
        self.send(b"E", fields)
        if self.db.in_transaction:
            self.failed = True

    def ready(self) -> None:
        status = b"E" if self.failed else (b"T" if self.db.in_transaction else b"I")
        self.send(b"Z", status)

    # -------------------------------------------------------------- startup
    def run(self) -> None:
        try:
            self._startup()
            self._loop()
        except (ConnectionError, OSError):
            pass
        finally:
            try:
                self.db.close()
                self.sock.close()
            except Exception:
                pass

    def _startup(self) -> None:
        while True:
            length = struct.unpack("!i", self.recv(4))[0]
            body = self.recv(length - 4)
            code = struct.unpack("!i", body[:4])[0]
            if code == 80877103:  # SSLRequest: refuse, continue in clear text
                self.sock.sendall(b"N")
                continue
            break
        kv = body[4:].split(b"\0")
        params = {kv[i].decode(): kv[i + 1].decode() for i in range(0, len(kv) - 1, 2) if kv[i]}
        srv = self.srv
        if params.get("user") != srv.user:
            return self.error(Exception(f'role "{params.get("user")}" does not exist'), "28000")
        if srv.auth == "password":
            self.send(b"R", struct.pack("!i", 3))
            if self._password_msg().rstrip(b"\0").decode() != srv.password:
                return self.error(Exception("password authentication failed"), "28P01")
        elif srv.auth == "md5":
            salt = os.urandom(4)
            self.send(b"R", struct.pack("!i", 5) + salt)
            inner = hashlib.md5((srv.password + srv.user).encode()).hexdigest().encode()
            if self._password_msg().rstrip(b"\0") != b"md5" + hashlib.md5(inner + salt).hexdigest().encode():
                return self.error(Exception("password authentication failed"), "28P01")
        elif srv.auth == "scram":
            if not self._scram():
                return self.error(Exception("password authentication failed"), "28P01")
        self.send(b"R", struct.pack("!i", 0))
        for k, v in (("server_version", "14.0 (dmcp fake)"), ("client_encoding", "UTF8"),
                     ("DateStyle", "ISO, MDY"), ("integer_datetimes", "on")):
            self.send(b"S", k.encode() + b"\0" + v.encode() + b"\0")
        self.send(b"K", struct.pack("!ii", os.getpid(), 1234))
        self.ready()

    def _password_msg(self) -> bytes:
        kind = self.recv(1)
        length = struct.unpack("!i", self.recv(4))[0]
        body = self.recv(length - 4)
        if kind != b"p":
            raise ConnectionError
        return body

    def _scram(self) -> bool:
        srv = self.srv
        self.send(b"R", struct.pack("!i", 10) + b"SCRAM-SHA-256\0\0")
        body = self._password_msg()
        mech_end = body.index(b"\0")
        first = body[mech_end + 5:].decode()
        assert first.startswith("n,,")
        first_bare = first[3:]
        cnonce = dict(kv.split("=", 1) for kv in first_bare.split(","))["r"]
        salt, iters = os.urandom(16), 4096
        nonce = cnonce + base64.b64encode(os.urandom(12)).decode()
        server_first = f"r={nonce},s={base64.b64encode(salt).decode()},i={iters}"
        self.send(b"R", struct.pack("!i", 11) + server_first.encode())
        final = self._password_msg().decode()
        attrs = dict(kv.split("=", 1) for kv in final.split(","))
        without_proof = final[:final.index(",p=")]
        auth_message = f"{first_bare},{server_first},{without_proof}"
        salted = hashlib.pbkdf2_hmac("sha256", srv.password.encode(), salt, iters)
        client_key = hmac.new(salted, b"Client Key", hashlib.sha256).digest()
        stored = hashlib.sha256(client_key).digest()
        sig = hmac.new(stored, auth_message.encode(), hashlib.sha256).digest()
        proof = base64.b64decode(attrs["p"])
        recovered = bytes(a ^ b for a, b in zip(proof, sig))
        if attrs.get("r") != nonce or hashlib.sha256(recovered).digest() != stored:
            return False
        server_key = hmac.new(salted, b"Server Key", hashlib.sha256).digest()
        ssig = hmac.new(server_key, auth_message.encode(), hashlib.sha256).digest()
        self.send(b"R", struct.pack("!i", 12) + b"v=" + base64.b64encode(ssig))
        return True

    # ------------------------------------------------------------ statements
    def _run_sql(self, sql: str, params: list) -> Tuple[list, list, str]:
        """(columns, rows, command tag) of one statement."""
        self.srv.statements.append(sql)
        text = sql.strip().rstrip(";").strip()
        head = text.split(None, 2)
        verb = head[0].upper() if head else ""
        if self.failed and verb not in ("ROLLBACK", "COMMIT"):
            raise _PgStateError("current transaction is aborted, commands ignored until end of transaction block")
        if verb == "SET" or (verb == "CREATE" and len(head) > 1 and head[1].upper() == "SCHEMA"):
            return [], [], "SET" if verb == "SET" else "CREATE SCHEMA"
        if verb in ("COMMIT", "END") and self.failed:
            self.db.execute("ROLLBACK")
            self.failed = False
            return [], [], "ROLLBACK"
        if verb == "ROLLBACK":
            self.failed = False
            if self.db.in_transaction:
                self.db.execute("ROLLBACK")
            return [], [], "ROLLBACK"
        m = re.match(r"(?is)ALTER\s+TABLE\s+(\w+)\s+ADD\s+COLUMN\s+IF\s+NOT\s+EXISTS\s+(.*)", text)
        if m:
            try:
                self.db.execute(f"ALTER TABLE {m.group(1)} ADD COLUMN {m.group(2)}")
            except sqlite3.OperationalError as e:
                if "duplicate column" not in str(e):
                    raise
            return [], [], "ALTER TABLE"
        cur = self.db.execute(_to_sqlite(text), params)
        cols = [d[0] for d in cur.description] if cur.description else []
        rows = cur.fetchall() if cols else []
        if verb == "SELECT" or cols:
            tag = f"SELECT {len(rows)}"
        elif verb == "INSERT":
            tag = f"INSERT 0 {cur.rowcount}"
        elif verb in ("UPDATE", "DELETE"):
            tag = f"{verb} {cur.rowcount}"
        else:
            tag = " ".join(head[:2]).upper() if len(head) > 1 else verb
        return cols, rows, tag

    def _row_description(self, cols: list, rows: list) -> bytes:
        out = [struct.pack("!h", len(cols))]
        for i, c in enumerate(cols):
            oid = 25
            for r in rows:
                v = r[i]
                if v is None:
                    continue
                oid = 20 if isinstance(v, int) else 701 if isinstance(v, float) else 25
                break
            out.append(c.encode() + b"\0" + struct.pack("!ihihih", 0, 0, oid, -1, -1, 0))
        return b"".join(out)

    def _send_rows(self, rows: list) -> None:
        for r in rows:
            parts = [struct.pack("!h", len(r))]
            for v in r:
                if v is None:
                    parts.append(struct.pack("!i", -1))
                else:
                    raw = (repr(v) if isinstance(v, float) else str(v)).encode("utf-8")
                    parts.append(struct.pack("!i", len(raw)) + raw)
            self.send(b"D", b"".join(parts))

    def _loop(self) -> None:
        while True:
            kind = self.recv(1)
            length = struct.unpack("!i", self.recv(4))[0]
            body = self.recv(length - 4)
            if kind == b"X":
                return
            if kind == b"S":
                self.skip = False
                self.ready()
                continue
            if self.skip:
                continue
            try:
                self._dispatch(kind, body)
            except Exception as e:  # noqa: BLE001 -- every failure becomes an ErrorResponse
                self.error(e, "25P02" if isinstance(e, _PgStateError) else None)
                if kind != b"Q":
                    self.skip = True
                else:
                    self.ready()

    def _dispatch(self, kind: bytes, body: bytes) -> None:
        if kind == b"Q":
            script = body.rstrip(b"\0").decode("utf-8")
            for stmt in [s for s in _split(script) if s.strip()]:
                cols, rows, tag = self._run_sql(stmt, [])
                if cols:
                    self.send(b"T", self._row_description(cols, rows))
                    self._send_rows(rows)
                self.send(b"C", tag.encode() + b"\0")
            self.ready()
        elif kind == b"P":
            name_end = body.index(b"\0")
            q_end = body.index(b"\0", name_end + 1)
            self.prepared[body[:name_end].decode()] = body[name_end + 1:q_end].decode("utf-8")
            self.send(b"1")
        elif kind == b"B":
            portal_end = body.index(b"\0")
            stmt_end = body.index(b"\0", portal_end + 1)
            stmt = body[portal_end + 1:stmt_end].decode()
            pos = stmt_end + 1
            nfmt = struct.unpack("!h", body[pos:pos + 2])[0]
            pos += 2 + 2 * nfmt
            nparams = struct.unpack("!h", body[pos:pos + 2])[0]
            pos += 2
            params = []
            for _ in range(nparams):
                ln = struct.unpack("!i", body[pos:pos + 4])[0]
                pos += 4
                if ln < 0:
                    params.append(None)
                else:
                    params.append(_param(body[pos:pos + ln]))
                    pos += ln
            if stmt not in self.prepared:
                raise _PgStateError(f'prepared statement "{stmt}" does not exist')
            self.portal = (self.prepared[stmt], params)
            self.result = None
            self.send(b"2")
        elif kind == b"D":
            if body[:1] == b"P":
                self.result = self._run_sql(*self.portal)
                cols, rows, _ = self.result
                if cols:
                    self.send(b"T", self._row_description(cols, rows))
                else:
                    self.send(b"n")
            else:
                self.send(b"t", struct.pack("!h", 0))
                self.send(b"n")
        elif kind == b"E":
            if self.result is None:
                self.result = self._run_sql(*self.portal)
            cols, rows, tag = self.result
            self._send_rows(rows)
            self.send(b"C", tag.encode() + b"\0")
            self.result = None
        elif kind == b"C":
            if body[:1] == b"S":
                self.prepared.pop(body[1:].rstrip(b"\0").decode(), None)
            self.send(b"3")
        elif kind == b"H":  # Flush
            pass
        else:
            raise _PgStateError(f"unsupported message {kind!r}")


class _PgStateError(Exception):
    pass


def _split(script: str) -> List[str]:
    out, buf, quote = [], [], False
    for ch in script:
        if ch == "'":
            quote = not quote
        if ch == ";" and not quote:
            out.append("".join(buf))
            buf = []
        else:
            buf.append(ch)
    if "".join(buf).strip():
        out.append("".join(buf))
    return out
