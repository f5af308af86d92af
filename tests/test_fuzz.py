"""Seeded mutation fuzzing of the hand-written native front-ends and the
loose-object reader.

The reference parses with JavaParser, Babel and go/ast, and isolates its one
native tool (the Go analyzer) in a subprocess with a 120 s kill
(``GoSourceParser.java:62, 339-418``).  dmcp runs its own C++ lexers, a zlib
inflater and the row builders inside the server process, so malformed input
must never crash it: every mutated file must produce valid JSON, and every
corrupted git object must come back as "not readable" (None), never a fault.

Corpus: the reference-derived fixtures of the parser tests (Java / TS / Go
sources shaped like ``JavaSourceParserTest``, ``NodeJsGraalParserTest`` and
``analyzer_test.go``) plus generated Spring / NestJS / gin projects.
Mutations: byte flips, syntax-character insertions, deletions, duplications,
truncations and splices between files.  ``DMCP_FUZZ_ITERS`` scales the run
(default 4,000 mutated files + 600 corrupted objects); under
scripts/asan_tests.sh the same test runs on the ASan/UBSan build.
"""
import json
import os
import random
import zlib

import pytest

from dmcp.utils import synth

ITERS = int(os.environ.get("DMCP_FUZZ_ITERS", "4000"))
SYNTAX = [b"{", b"}", b"(", b")", b"[", b"]", b"<", b">", b"\"", b"'", b"`", b"/*", b"*/", b"//", b"@", b";", b",",
          b".", b"\\", b"\n", b"${", b"=>", b"...", b"::", b"#", b"\x00", b"\xff", b"\xc3", b"func ", b"class ",
          b"import ", b"package ", b"@Get(", b"export ", b"interface ", b"struct {", b"go ", b"r`", b"\"\"\""]

JAVA_FIXTURES = [
    b"""package co.fanki.user;

import co.fanki.order.Order;
import static co.fanki.util.Strings.isBlank;
import java.util.*;

@RestController
@RequestMapping("/api/users")
public class UserController {
    private final UserService service;

    public UserController(UserService service) { this.service = service; }

    @GetMapping("/{id}")
    public User get(@PathVariable String id) throws NotFoundException { return service.find(id); }

    @RequestMapping(value = "/search", method = RequestMethod.POST)
    public List<User> search(SearchRequest req, Order... orders) { return List.of(); }

    public record Page<T>(List<T> items, int total) {}
}
""",
    b"""package co.fanki.order;

@Service
public class OrderService implements Handler<Order> {
    @KafkaListener(topics = {"a", "b"})
    public void on(Order o) { if (o == null) throw new IllegalStateException("x"); }
    static class Inner { void x() { String s = "}"; char c = '{'; } }
    /* unterminated? no */ int[] arr = new int[]{1, 2};
    String text = \"\"\"
        a text block with "quotes" and } braces
        \"\"\";
}
""",
]
TS_FIXTURES = [
    b"""import { Controller, Get, Post, Body, Param } from '@nestjs/common';
import * as svc from './users.service';
import Default, { named as alias } from '../shared/util';

@Controller('users')
export class UsersController {
  constructor(private readonly service: svc.UsersService) {}
  @Get(':id')
  findOne(@Param('id') id: string): Promise<User> { return this.service.find(id); }
  @Post()
  create = async (@Body() dto: CreateUserDto) => this.service.create(dto);
}
export const handler = useCallback((e: Event) => { const t = `a ${e.type} b`; }, []);
export async function GET(req: Request) { return new Response(JSON.stringify({ a: /re}gex/g })); }
""",
    b"""const express = require('express');
const router = express.Router();
router.get('/orders/:id', async (req, res) => { res.json({ id: req.params.id }); });
app.post("/pay", (req, res) => res.send(<div className="x">{`tpl`}</div>));
export default { method() { return 1 }, arrow: () => 2 };
""",
]
GO_FIXTURES = [
    b"""package handler

import (
\t"net/http"
\tsvc "github.com/acme/app/internal/service"
\t"github.com/gin-gonic/gin"
)

// Handler serves orders.
type Handler struct {
\tsvc *svc.Service
\tmodel.Base
}

func (h *Handler) Get(c *gin.Context) { if c == nil { panic("nil") } }

func Serve(w http.ResponseWriter, r *http.Request) { _ = `raw ` + "str" }

func main() { r := gin.Default(); r.GET("/x", nil); r.Group("/v1") }
""",
]


def _corpus(tmp_path):
    java, ts, go = list(JAVA_FIXTURES), list(TS_FIXTURES), list(GO_FIXTURES)
    for gen, out, ext in ((lambda r: synth.java_spring_repo(r, 24, commit=False), java, ".java"),
                          (lambda r: synth.nestjs_repo(r, 3, commit=False), ts, ".ts"),
                          (lambda r: synth.go_gin_repo(r, 2, commit=False), go, ".go")):
        root = str(tmp_path / ext[1:])
        gen(root)
        for d, _, files in os.walk(root):
            for f in files:
                if f.endswith(ext):
                    with open(os.path.join(d, f), "rb") as fh:
                        out.append(fh.read())
    return {"java": java, "typescript": ts, "go": go}


def _mutate(rnd: random.Random, data: bytes, pool) -> bytes:
    b = bytearray(data)
    for _ in range(rnd.randint(1, 6)):
        op = rnd.randrange(6)
        pos = rnd.randrange(len(b) + 1) if b else 0
        if op == 0 and b:  # flip
            i = rnd.randrange(len(b))
            b[i] ^= 1 << rnd.randrange(8)
        elif op == 1:  # insert syntax
            b[pos:pos] = rnd.choice(SYNTAX)
        elif op == 2 and b:  # delete a range
            del b[pos:pos + rnd.randint(1, 40)]
        elif op == 3 and b:  # duplicate a range
            seg = b[pos:pos + rnd.randint(1, 80)]
            b[pos:pos] = seg
        elif op == 4:  # truncate
            del b[pos:]
        else:  # splice another file's head
            other = rnd.choice(pool)
            b[pos:] = other[:rnd.randint(0, len(other))]
    return bytes(b)


@pytest.fixture(scope="module")
def native():
    from dmcp.parsers.base import native as nat
    return nat()


def test_fuzz_front_ends_never_crash(native, tmp_path):
    rnd = random.Random(1234)
    corpus = _corpus(tmp_path)
    langs = list(corpus)
    n_json = 0
    for it in range(ITERS):
        lang = langs[it % 3]
        src = _mutate(rnd, rnd.choice(corpus[lang]), corpus[lang])
        if lang == "go":
            out = native.scan_sources([("go.mod", b"module github.com/acme/app\n\ngo 1.22\n"),
                                       (f"internal/p{it % 7}/x.go", src), ("cmd/main.go", corpus["go"][0])], "go")
        else:
            path = f"src/main/java/co/x/F{it}.java" if lang == "java" else f"src/f{it}.ts"
            out = native.analyze_source(src.decode("utf-8", "replace"), lang, path, "nestjs" if it % 2 else "unknown")
        json.loads(out)
        n_json += 1
    assert n_json == ITERS


def _loose(objdir, body: bytes, kind: bytes) -> str:
    import hashlib
    raw = kind + b" " + str(len(body)).encode() + b"\0" + body
    sha = hashlib.sha1(raw).hexdigest()
    d = os.path.join(objdir, sha[:2])
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, sha[2:]), "wb") as f:
        f.write(zlib.compress(raw))
    return sha


def test_fuzz_corrupted_loose_objects(native, tmp_path):
    from dmcp import _srcscan
    rnd = random.Random(99)
    objdir = str(tmp_path / "objects")
    blob = _loose(objdir, b"class A {}\n" * 50, b"blob")
    tree_body = b"100644 A.java\0" + bytes.fromhex(blob)
    tree = _loose(objdir, tree_body, b"tree")
    commit = _loose(objdir, b"tree " + tree.encode() + b"\nauthor a <a> 1 +0000\n\nmsg\n", b"commit")
    assert _srcscan.read_loose_blobs([objdir], [blob])[0][0] == b"class A {}\n" * 50
    assert _srcscan.list_tree_loose([objdir], commit) == [("A.java", blob)]
    files = {s: os.path.join(objdir, s[:2], s[2:]) for s in (blob, tree, commit)}
    originals = {s: open(p, "rb").read() for s, p in files.items()}
    iters = max(200, ITERS // 7)
    for it in range(iters):
        sha = rnd.choice(list(files))
        raw = zlib.decompress(originals[sha])
        op = rnd.randrange(5)
        if op == 0:    # corrupt the zlib stream itself
            data = bytearray(originals[sha])
            for _ in range(rnd.randint(1, 4)):
                data[rnd.randrange(len(data))] ^= 1 << rnd.randrange(8)
            data = bytes(data)
        elif op == 1:  # truncated stream
            data = originals[sha][:rnd.randrange(len(originals[sha]))]
        else:          # a valid stream of a corrupted object (header / size / body / tree entries)
            b = bytearray(raw)
            if op == 2:
                hdr = raw.index(b"\0")
                b[rnd.randrange(hdr + 1)] = rnd.choice(b" 0123456789\0xz")
            elif op == 3:
                del b[rnd.randrange(len(b)):]
            else:
                for _ in range(rnd.randint(1, 6)):
                    b[rnd.randrange(len(b))] = rnd.randrange(256)
            data = zlib.compress(bytes(b))
        with open(files[sha], "wb") as f:
            f.write(data)
        got, _ = _srcscan.read_loose_blobs([objdir], [blob], 1, 1 << 20)
        assert got[0] is None or isinstance(got[0], bytes)
        lt = _srcscan.list_tree_loose([objdir], commit)
        assert lt is None or isinstance(lt, list)
        with open(files[sha], "wb") as f:
            f.write(originals[sha])
    assert _srcscan.list_tree_loose([objdir], commit) == [("A.java", blob)]


def test_native_module_is_the_requested_build():
    """Under scripts/asan_tests.sh the instrumented module must be the one
    loaded (DMCP_SRCSCAN_SO), not the release build next to the package."""
    from dmcp import _srcscan
    want = os.environ.get("DMCP_SRCSCAN_SO")
    if want:
        assert os.path.samefile(_srcscan.__file__, want)
    else:
        assert os.path.dirname(_srcscan.__file__).endswith("dmcp")
