"""PostgreSQL frontend/backend protocol (v3) client -- no driver dependency.

The reference persists to PostgreSQL through Hikari + JDBI
(``application.yml:11-29``, ``config/DatabaseConfiguration.java:37-52``).
No PostgreSQL driver is installed on this host (no psycopg / asyncpg), so the
PostgreSQL store (:mod:`dmcp.store.pg`) talks the wire protocol itself:

* startup with ``user`` / ``database`` / ``application_name``, optional TLS
  (``SSLRequest``; ``sslmode`` disable / prefer / require),
* authentication: trust, cleartext, MD5 and SCRAM-SHA-256 (RFC 5802 / 7677,
  server signature verified),
* the extended query protocol with text-format parameters and results
  (Parse / Bind / Describe / Execute / Sync), named prepared statements
  cached per SQL text, and pipelined ``executemany`` (one Parse, a Bind /
  Execute pair per row, one Sync per chunk -- no round trip per row),
* the simple query protocol for multi-statement scripts (migrations),
* result decoding by type OID (bool, int2/4/8, float4/8, numeric, json(b) as
  text, timestamps normalised to ISO-8601), rows addressable by index and by
  column name like ``sqlite3.Row``.

A connection is used by one thread at a time (:class:`dmcp.store.pg.PgDatabase`
keeps one per thread).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import re
import socket
import ssl
import struct
from collections import OrderedDict
from datetime import date, datetime
from typing import Any, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

PROTOCOL_V3 = 196608
SSL_REQUEST_CODE = 80877103

# type OIDs decoded from text format
_INT_OIDS = {20, 21, 23, 26}
_FLOAT_OIDS = {700, 701}
_BOOL_OID = 16
_NUMERIC_OID = 1700
_TS_OIDS = {1114, 1184}


class PgError(Exception):
    """An ErrorResponse from the server (or a protocol failure)."""

    def __init__(self, message: str, sqlstate: str = "", fields: Optional[Dict[str, str]] = None) -> None:
        super().__init__(f"{sqlstate}: {message}" if sqlstate else message)
        self.sqlstate = sqlstate
        self.fields = fields or {}

    @property
    def is_unique_violation(self) -> bool:
        return self.sqlstate == "23505"


class PgRow(tuple):
    """A result row: ``row[i]`` and ``row["column"]`` (as ``sqlite3.Row``)."""

    _index: Dict[str, int]

    def __new__(cls, values: Sequence[Any], index: Dict[str, int]) -> "PgRow":
        r = super().__new__(cls, values)
        r._index = index
        return r

    def __getitem__(self, key):  # type: ignore[override]
        if isinstance(key, str):
            try:
                return tuple.__getitem__(self, self._index[key])
            except KeyError:
                raise IndexError(f"no such column: {key}") from None
        return tuple.__getitem__(self, key)

    def keys(self) -> List[str]:
        return list(self._index)


class PgCursor:
    """Result of one statement: rows, ``rowcount`` and ``description``."""

    def __init__(self, rows: List[PgRow], rowcount: int, columns: List[str], tag: str) -> None:
        self._rows = rows
        self._pos = 0
        self.rowcount = rowcount
        self.description = [(c, None, None, None, None, None, None) for c in columns] if columns else None
        self.command_tag = tag

    def fetchone(self) -> Optional[PgRow]:
        if self._pos >= len(self._rows):
            return None
        r = self._rows[self._pos]
        self._pos += 1
        return r

    def fetchall(self) -> List[PgRow]:
        out = self._rows[self._pos:]
        self._pos = len(self._rows)
        return out

    def __iter__(self) -> Iterator[PgRow]:
        while True:
            r = self.fetchone()
            if r is None:
                return
            yield r


_QMARK = re.compile(r"'(?:[^']|'')*'|\"(?:[^\"]|\"\")*\"|\?")


def qmark_to_dollar(sql: str) -> str:
    """``?`` placeholders (the repositories' SQLite style) -> ``$1..$n``;
    question marks inside quoted literals / identifiers are left alone."""
    n = 0

    def sub(m: "re.Match[str]") -> str:
        nonlocal n
        if m.group(0) != "?":
            return m.group(0)
        n += 1
        return f"${n}"
    return _QMARK.sub(sub, sql)


def _encode_param(v: Any) -> Optional[bytes]:
    if v is None:
        return None
    if isinstance(v, bool):
        return b"t" if v else b"f"
    if isinstance(v, (int, float)):
        return repr(v).encode()
    if isinstance(v, (datetime, date)):
        return v.isoformat().encode()
    if isinstance(v, (bytes, bytearray, memoryview)):
        return b"\\x" + bytes(v).hex().encode()
    return str(v).encode("utf-8")


def _decode(oid: int, raw: bytes) -> Any:
    if oid in _INT_OIDS:
        return int(raw)
    if oid in _FLOAT_OIDS:
        return float(raw)
    if oid == _BOOL_OID:
        return raw == b"t"
    if oid == _NUMERIC_OID:
        s = raw.decode()
        try:
            return int(s)
        except ValueError:
            return float(s)
    s = raw.decode("utf-8")
    if oid in _TS_OIDS:
        # '2026-10-16 12:00:00.123+00' -> '2026-10-16T12:00:00.123+00:00'
        s = s.replace(" ", "T", 1)
        if len(s) >= 3 and s[-3] in "+-" and s[-2:].isdigit():
            s += ":00"
    return s


class PgConnection:
    """One PostgreSQL session over TCP (or a Unix socket path as ``host``)."""

    STATEMENT_CACHE = 256
    PIPELINE_ROWS = 1000

    def __init__(self, host: str = "127.0.0.1", port: int = 5432, user: str = "postgres",
                 password: Optional[str] = None, database: Optional[str] = None, sslmode: str = "prefer",
                 connect_timeout: float = 10.0, application_name: str = "dmcp",
                 options: Optional[Dict[str, str]] = None) -> None:
        self.user = user
        self.password = password or ""
        self.server_params: Dict[str, str] = {}
        self.tx_status = "I"
        self._stmts: "OrderedDict[str, str]" = OrderedDict()
        self._stmt_seq = 0
        self._buf = b""
        if host.startswith("/"):
            sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            sock.settimeout(connect_timeout)
            sock.connect(os.path.join(host, f".s.PGSQL.{port}"))
        else:
            sock = socket.create_connection((host, port), timeout=connect_timeout)
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        sock.settimeout(None)
        self._sock = sock
        if sslmode != "disable" and not host.startswith("/"):
            self._sock.sendall(struct.pack("!ii", 8, SSL_REQUEST_CODE))
            answer = self._recv_exact(1)
            if answer == b"S":
                ctx = ssl.create_default_context()
                if sslmode in ("prefer", "require"):  # libpq semantics: encrypt, do not verify
                    ctx.check_hostname = False
                    ctx.verify_mode = ssl.CERT_NONE
                self._sock = ctx.wrap_socket(self._sock, server_hostname=host)
            elif sslmode in ("require", "verify-ca", "verify-full"):
                raise PgError("server does not support TLS (sslmode=%s)" % sslmode)
        params = {"user": user, "database": database or user, "application_name": application_name,
                  "client_encoding": "UTF8", "DateStyle": "ISO"}
        params.update(options or {})
        body = struct.pack("!i", PROTOCOL_V3) + b"".join(
            k.encode() + b"\0" + str(v).encode() + b"\0" for k, v in params.items()) + b"\0"
        self._sock.sendall(struct.pack("!i", len(body) + 4) + body)
        self._authenticate()
        self._read_until_ready()

    # ------------------------------------------------------------ transport
    def _recv_exact(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self._sock.recv(max(65536, n - len(self._buf)))
            if not chunk:
                raise PgError("connection closed by the server")
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def _read_msg(self) -> Tuple[bytes, bytes]:
        head = self._recv_exact(5)
        kind, length = head[:1], struct.unpack("!i", head[1:])[0]
        return kind, self._recv_exact(length - 4)

    @staticmethod
    def _msg(kind: bytes, body: bytes = b"") -> bytes:
        return kind + struct.pack("!i", len(body) + 4) + body

    def _send(self, data: bytes) -> None:
        self._sock.sendall(data)

    # ------------------------------------------------------- authentication
    def _authenticate(self) -> None:
        scram = None
        while True:
            kind, body = self._read_msg()
            if kind == b"E":
                raise self._error(body)
            if kind != b"R":
                raise PgError(f"unexpected message {kind!r} during authentication")
            code = struct.unpack("!i", body[:4])[0]
            if code == 0:
                return
            if code == 3:  # cleartext
                self._send(self._msg(b"p", self.password.encode() + b"\0"))
            elif code == 5:  # MD5: "md5" + md5(md5(password + user) + salt)
                salt = body[4:8]
                inner = hashlib.md5((self.password + self.user).encode()).hexdigest().encode()
                digest = b"md5" + hashlib.md5(inner + salt).hexdigest().encode()
                self._send(self._msg(b"p", digest + b"\0"))
            elif code == 10:  # SASL: mechanisms
                mechs = [m for m in body[4:].split(b"\0") if m]
                if b"SCRAM-SHA-256" not in mechs:
                    raise PgError(f"no supported SASL mechanism in {mechs}")
                scram = _Scram(self.password)
                first = scram.client_first().encode()
                self._send(self._msg(b"p", b"SCRAM-SHA-256\0" + struct.pack("!i", len(first)) + first))
            elif code == 11:  # SASL continue
                if scram is None:
                    raise PgError("SASL continue without a started exchange")
                self._send(self._msg(b"p", scram.client_final(body[4:].decode()).encode()))
            elif code == 12:  # SASL final: verify the server signature
                if scram is None or not scram.verify(body[4:].decode()):
                    raise PgError("SCRAM server signature mismatch")
            else:
                raise PgError(f"unsupported authentication request {code}")

    # -------------------------------------------------------------- results
    @staticmethod
    def _error(body: bytes) -> PgError:
        fields: Dict[str, str] = {}
        for part in body.split(b"\0"):
            if part:
                fields[chr(part[0])] = part[1:].decode("utf-8", "replace")
        return PgError(fields.get("M", "server error"), fields.get("C", ""), fields)

    def _read_until_ready(self) -> None:
        err = None
        while True:
            kind, body = self._read_msg()
            if kind == b"Z":
                self.tx_status = body[:1].decode()
                break
            if kind == b"E":
                err = err or self._error(body)
            elif kind == b"S":
                k, v = body.split(b"\0")[:2]
                self.server_params[k.decode()] = v.decode()
        if err is not None:
            raise err

    def _collect(self, n_results: int) -> List[PgCursor]:
        """Reads ``n_results`` statement results up to ReadyForQuery."""
        out: List[PgCursor] = []
        cols: List[str] = []
        oids: List[int] = []
        index: Dict[str, int] = {}
        rows: List[PgRow] = []
        err: Optional[PgError] = None
        while True:
            kind, body = self._read_msg()
            if kind == b"D":
                n = struct.unpack("!h", body[:2])[0]
                pos = 2
                vals = []
                for i in range(n):
                    ln = struct.unpack("!i", body[pos:pos + 4])[0]
                    pos += 4
                    if ln < 0:
                        vals.append(None)
                    else:
                        vals.append(_decode(oids[i], body[pos:pos + ln]))
                        pos += ln
                rows.append(PgRow(vals, index))
            elif kind == b"T":
                n = struct.unpack("!h", body[:2])[0]
                pos = 2
                cols, oids = [], []
                for _ in range(n):
                    end = body.index(b"\0", pos)
                    cols.append(body[pos:end].decode())
                    pos = end + 1
                    oids.append(struct.unpack("!i", body[pos + 6:pos + 10])[0])
                    pos += 18
                index = {c: i for i, c in enumerate(cols)}
                rows = []
            elif kind == b"C":
                tag = body[:-1].decode()
                parts = tag.split()
                count = int(parts[-1]) if parts and parts[-1].isdigit() else -1
                out.append(PgCursor(rows, count, cols, tag))
                cols, oids, index, rows = [], [], {}, []
            elif kind == b"I":  # empty query
                out.append(PgCursor([], -1, [], ""))
            elif kind == b"E":
                err = err or self._error(body)
            elif kind == b"Z":
                self.tx_status = body[:1].decode()
                break
            elif kind == b"S":
                k, v = body.split(b"\0")[:2]
                self.server_params[k.decode()] = v.decode()
            # '1' ParseComplete, '2' BindComplete, 'n' NoData, 'N' notices,
            # 's' PortalSuspended, 'A' notifications: nothing to keep
        if err is not None:
            raise err
        return out

    # ------------------------------------------------------------ statements
    def _prepare(self, sql: str) -> Tuple[str, bytes]:
        """(statement name, Parse message or b"" when already prepared)."""
        name = self._stmts.get(sql)
        if name is not None:
            self._stmts.move_to_end(sql)
            return name, b""
        self._stmt_seq += 1
        name = f"dmcp_{self._stmt_seq}"
        parse = self._msg(b"P", name.encode() + b"\0" + sql.encode() + b"\0" + struct.pack("!h", 0))
        return name, parse

    def _remember(self, sql: str, name: str) -> bytes:
        """Caches a prepared statement; returns Close messages for evictions."""
        self._stmts[sql] = name
        closes = b""
        while len(self._stmts) > self.STATEMENT_CACHE:
            _, old = self._stmts.popitem(last=False)
            closes += self._msg(b"C", b"S" + old.encode() + b"\0")
        return closes

    @classmethod
    def _bind(cls, name: str, params: Sequence[Any]) -> bytes:
        """Bind the unnamed portal to statement ``name``: text parameters, text results."""
        parts = [b"\0", name.encode(), b"\0", struct.pack("!hh", 0, len(params))]
        for p in params:
            raw = _encode_param(p)
            if raw is None:
                parts.append(struct.pack("!i", -1))
            else:
                parts.append(struct.pack("!i", len(raw)))
                parts.append(raw)
        parts.append(struct.pack("!h", 0))
        return cls._msg(b"B", b"".join(parts))

    _DESCRIBE_PORTAL = b"D" + struct.pack("!i", 6) + b"P\0"
    _EXECUTE_ALL = b"E" + struct.pack("!i", 9) + b"\0" + struct.pack("!i", 0)
    _SYNC = b"S" + struct.pack("!i", 4)

    def _discard(self, name: str) -> None:
        """Closes a statement whose Parse may or may not have succeeded
        (closing a missing statement is not an error)."""
        self._send(self._msg(b"C", b"S" + name.encode() + b"\0") + self._SYNC)
        try:
            self._collect(0)
        except PgError:
            pass

    def _statement_done(self, sql: str, name: str, parsed: bool, ok: bool) -> None:
        if not parsed:
            return
        if not ok:
            self._discard(name)
            return
        closes = self._remember(sql, name)
        if closes:
            self._send(closes + self._SYNC)
            self._collect(0)

    def execute(self, sql: str, params: Sequence[Any] = ()) -> PgCursor:
        """One statement with ``$n`` (or ``?``) placeholders."""
        if "?" in sql:
            sql = qmark_to_dollar(sql)
        name, parse = self._prepare(sql)
        self._send(parse + self._bind(name, params) + self._DESCRIBE_PORTAL + self._EXECUTE_ALL + self._SYNC)
        ok = False
        try:
            res = self._collect(1)
            ok = True
        finally:
            self._statement_done(sql, name, bool(parse), ok)
        return res[0] if res else PgCursor([], -1, [], "")

    def executemany(self, sql: str, seq: Iterable[Sequence[Any]]) -> PgCursor:
        """One Parse, then Bind/Execute per row, pipelined in chunks."""
        if "?" in sql:
            sql = qmark_to_dollar(sql)
        total = 0
        rows = iter(seq)
        while True:
            chunk = []
            for p in rows:
                chunk.append(p)
                if len(chunk) >= self.PIPELINE_ROWS:
                    break
            if not chunk:
                break
            name, parse = self._prepare(sql)
            msg = [parse] + [self._bind(name, p) + self._EXECUTE_ALL for p in chunk] + [self._SYNC]
            self._send(b"".join(msg))
            ok = False
            try:
                res = self._collect(len(chunk))
                ok = True
            finally:
                self._statement_done(sql, name, bool(parse), ok)
            total += sum(max(0, c.rowcount) for c in res)
            if len(chunk) < self.PIPELINE_ROWS:
                break
        return PgCursor([], total, [], "")

    def execute_script(self, script: str) -> List[PgCursor]:
        """Simple-query protocol: several ``;``-separated statements, no parameters."""
        self._send(self._msg(b"Q", script.encode("utf-8") + b"\0"))
        return self._collect(0)

    def close(self) -> None:
        try:
            self._send(self._msg(b"X"))
        except OSError:
            pass
        try:
            self._sock.close()
        except OSError:
            pass


class _Scram:
    """SCRAM-SHA-256 client (channel binding not used: gs2 header ``n,,``)."""

    def __init__(self, password: str) -> None:
        self.password = password
        self.nonce = base64.b64encode(os.urandom(18)).decode()
        self.first_bare = f"n=,r={self.nonce}"
        self.auth_message = ""
        self.salted = b""

    def client_first(self) -> str:
        return "n,," + self.first_bare

    def client_final(self, server_first: str) -> str:
        attrs = dict(kv.split("=", 1) for kv in server_first.split(","))
        rnonce, salt, iters = attrs["r"], base64.b64decode(attrs["s"]), int(attrs["i"])
        if not rnonce.startswith(self.nonce):
            raise PgError("SCRAM server nonce does not extend the client nonce")
        self.salted = hashlib.pbkdf2_hmac("sha256", self.password.encode(), salt, iters)
        client_key = hmac.new(self.salted, b"Client Key", hashlib.sha256).digest()
        stored_key = hashlib.sha256(client_key).digest()
        without_proof = f"c=biws,r={rnonce}"
        self.auth_message = f"{self.first_bare},{server_first},{without_proof}"
        sig = hmac.new(stored_key, self.auth_message.encode(), hashlib.sha256).digest()
        proof = bytes(a ^ b for a, b in zip(client_key, sig))
        return f"{without_proof},p={base64.b64encode(proof).decode()}"

    def verify(self, server_final: str) -> bool:
        attrs = dict(kv.split("=", 1) for kv in server_final.split(","))
        server_key = hmac.new(self.salted, b"Server Key", hashlib.sha256).digest()
        expected = hmac.new(server_key, self.auth_message.encode(), hashlib.sha256).digest()
        return hmac.compare_digest(base64.b64decode(attrs.get("v", "")), expected)
