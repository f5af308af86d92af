"""Deterministic synthetic repositories for benchmarks and tests.

There is no network on this host, so the BASELINE configs (a toy Spring
repo, a ~200-class Java monorepo, a NestJS service, a Go gin service) are
generated: realistic layering (controller -> service -> repository -> entity,
DTOs, exceptions, configuration), annotations, endpoints, parameter types
and cross-module imports, committed to a local git repository so the real
clone -> parse -> persist pipeline runs end to end.
"""
from __future__ import annotations

import os
import random
import subprocess
from typing import List, Optional

_DOMAINS = ["order", "user", "payment", "invoice", "ticket", "event", "venue", "seat", "fan", "refund",
            "coupon", "cart", "shipment", "catalog", "price", "review", "report", "audit", "notification",
            "session", "account", "wallet", "transfer", "ledger", "policy", "claim", "quote", "stock",
            "supplier", "warehouse"]
_VERBS = ["find", "create", "update", "delete", "list", "search", "validate", "approve", "cancel", "sync",
          "compute", "publish", "archive", "restore", "notify"]


def _cap(s: str) -> str:
    return s[:1].upper() + s[1:]


def _git_commit(root: str, message: str = "synthetic") -> str:
    env = dict(os.environ, GIT_AUTHOR_NAME="synth", GIT_AUTHOR_EMAIL="synth@local",
               GIT_COMMITTER_NAME="synth", GIT_COMMITTER_EMAIL="synth@local")
    if not os.path.isdir(os.path.join(root, ".git")):
        subprocess.run(["git", "init", "-q", "-b", "main", root], check=True, env=env)
    subprocess.run(["git", "-C", root, "add", "-A"], check=True, env=env)
    subprocess.run(["git", "-C", root, "commit", "-q", "--allow-empty", "-m", message], check=True, env=env)
    return subprocess.run(["git", "-C", root, "rev-parse", "HEAD"], check=True, env=env,
                          stdout=subprocess.PIPE, text=True).stdout.strip()


def _write(path: str, text: str) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", encoding="utf-8") as f:
        f.write(text)


def java_spring_repo(root: str, n_classes: int = 200, base_package: str = "co.acme.shop", seed: int = 7,
                     commit: bool = True, readme: bool = True) -> List[str]:
    """Writes a Spring Boot style repo with ~``n_classes`` classes; returns FQCNs."""
    rnd = random.Random(seed)
    kinds = ["Controller", "Service", "Repository", "Entity", "Request", "Response", "Exception", "Config"]
    per_domain = len(kinds)
    n_domains = max(1, (n_classes + per_domain - 1) // per_domain)
    fqcns: List[str] = []
    src = os.path.join(root, "src", "main", "java", *base_package.split("."))
    domains = []
    for d in range(n_domains):
        name = _DOMAINS[d % len(_DOMAINS)] + ("" if d < len(_DOMAINS) else str(d // len(_DOMAINS)))
        domains.append(name)
    count = 0
    for di, dom in enumerate(domains):
        D = _cap(dom)
        pkg = f"{base_package}.{dom}"
        other = domains[(di + 1) % len(domains)]
        O = _cap(other)
        files = {}
        files["Entity"] = f"""package {pkg};

import jakarta.persistence.Entity;
import jakarta.persistence.Id;
import java.time.Instant;

/** {D} aggregate. */
@Entity
public class {D} {{

    @Id
    private String id;
    private String name;
    private long amountCents;
    private Instant createdAt;

    public {D}() {{
    }}

    public {D}(String id, String name) {{
        this.id = id;
        this.name = name;
        this.createdAt = Instant.now();
    }}

    public String getId() {{ return id; }}

    public String getName() {{ return name; }}

    public long getAmountCents() {{ return amountCents; }}

    public void rename(final String newName) {{
        if (newName == null || newName.isBlank()) {{
            throw new IllegalArgumentException("name required");
        }}
        this.name = newName;
    }}
}}
"""
        files["Request"] = f"""package {pkg};

import java.util.List;

public record {D}Request(String name, long amountCents, List<String> tags) {{
    public {D}Request {{
        tags = tags == null ? List.of() : tags;
    }}

    public boolean hasTags() {{
        return !tags.isEmpty();
    }}
}}
"""
        files["Response"] = f"""package {pkg};

public class {D}Response {{
    private final String id;
    private final String name;

    public {D}Response(String id, String name) {{
        this.id = id;
        this.name = name;
    }}

    public static {D}Response from({D} entity) {{
        return new {D}Response(entity.getId(), entity.getName());
    }}

    public String id() {{ return id; }}
}}
"""
        files["Exception"] = f"""package {pkg};

public class {D}NotFoundException extends RuntimeException {{
    public {D}NotFoundException(String id) {{
        super("{dom} not found: " + id);
    }}
}}
"""
        files["Repository"] = f"""package {pkg};

import java.util.List;
import java.util.Optional;
import org.springframework.stereotype.Repository;

@Repository
public class {D}Repository {{

    private final java.util.Map<String, {D}> store = new java.util.concurrent.ConcurrentHashMap<>();

    public Optional<{D}> findById(String id) {{
        return Optional.ofNullable(store.get(id));
    }}

    public List<{D}> findAll() {{
        return List.copyOf(store.values());
    }}

    public {D} save({D} entity) {{
        store.put(entity.getId(), entity);
        return entity;
    }}

    public void delete(String id) {{
        store.remove(id);
    }}
}}
"""
        verbs = rnd.sample(_VERBS, 4)
        svc_methods = "\n".join(f"""
    public {D}Response {v}{D}(final {D}Request request, String id) throws {D}NotFoundException {{
        {D} entity = repository.findById(id).orElseThrow(() -> new {D}NotFoundException(id));
        entity.rename(request.name());
        {other}Service.touch(id);
        return {D}Response.from(repository.save(entity));
    }}""" for v in verbs)
        files["Service"] = f"""package {pkg};

import {base_package}.{other}.{O}Service;
import java.util.List;
import org.springframework.stereotype.Service;
import org.springframework.transaction.annotation.Transactional;

/**
 * Business rules for {dom}s.
 */
@Service
public class {D}Service {{

    private final {D}Repository repository;
    private final {O}Service {other}Service;

    public {D}Service({D}Repository repository, {O}Service {other}Service) {{
        this.repository = repository;
        this.{other}Service = {other}Service;
    }}

    @Transactional
    public List<{D}Response> list() {{
        return repository.findAll().stream().map({D}Response::from).toList();
    }}
{svc_methods}

    public void touch(String id) {{
        // audit hook
    }}
}}
"""
        ctrl_methods = "\n".join(f"""
    @{m}Mapping("/{v}/{{id}}")
    public {D}Response {v}(@PathVariable String id, @RequestBody {D}Request request) {{
        return service.{v}{D}(request, id);
    }}""" for m, v in zip(["Post", "Put", "Patch", "Delete"], verbs))
        files["Controller"] = f"""package {pkg};

import java.util.List;
import org.springframework.web.bind.annotation.*;

@RestController
@RequestMapping("/api/{dom}s")
public class {D}Controller {{

    private final {D}Service service;

    public {D}Controller({D}Service service) {{
        this.service = service;
    }}

    @GetMapping("/")
    public List<{D}Response> list() {{
        return service.list();
    }}
{ctrl_methods}
}}
"""
        files["Config"] = f"""package {pkg};

import org.springframework.context.annotation.Bean;
import org.springframework.context.annotation.Configuration;
import org.springframework.kafka.annotation.KafkaListener;

@Configuration
public class {D}Config {{

    @Bean
    public {D}Repository {dom}Repository() {{
        return new {D}Repository();
    }}

    @KafkaListener(topics = "{dom}-events")
    public void on{D}Event(String payload) {{
    }}
}}
"""
        names = {"Entity": D, "Request": f"{D}Request", "Response": f"{D}Response",
                 "Exception": f"{D}NotFoundException", "Repository": f"{D}Repository",
                 "Service": f"{D}Service", "Controller": f"{D}Controller", "Config": f"{D}Config"}
        for kind in kinds:
            if count >= n_classes:
                break
            _write(os.path.join(src, dom, names[kind] + ".java"), files[kind])
            fqcns.append(f"{pkg}.{names[kind]}")
            count += 1
    app_pkg = base_package
    _write(os.path.join(src, "Application.java"), f"""package {app_pkg};

import org.springframework.boot.autoconfigure.SpringBootApplication;

@SpringBootApplication
public class Application {{
    public static void main(String[] args) {{
    }}
}}
""")
    fqcns.append(f"{app_pkg}.Application")
    _write(os.path.join(root, "pom.xml"), "<project><modelVersion>4.0.0</modelVersion></project>\n")
    if readme:
        _write(os.path.join(root, "README.md"), f"# {os.path.basename(root)}\n\nSynthetic commerce platform "
               f"with {len(domains)} business domains ({', '.join(domains[:6])}...).\n")
    if commit:
        _git_commit(root)
    return fqcns


def nestjs_repo(root: str, n_modules: int = 10, seed: int = 3, commit: bool = True) -> List[str]:
    rnd = random.Random(seed)
    idents = []
    _write(os.path.join(root, "package.json"),
           '{"name":"svc","dependencies":{"@nestjs/core":"^10.0.0","@nestjs/common":"^10.0.0"},'
           '"devDependencies":{"typescript":"^5.4.0"}}\n')
    _write(os.path.join(root, "src", "main.ts"), "import { NestFactory } from '@nestjs/core';\n"
           "import { AppModule } from './app.module';\n\nasync function bootstrap() {\n"
           "  const app = await NestFactory.create(AppModule);\n  await app.listen(3000);\n}\nbootstrap();\n")
    _write(os.path.join(root, "src", "app.module.ts"), "import { Module } from '@nestjs/common';\n\n"
           "@Module({})\nexport class AppModule {}\n")
    idents += ["main", "app.module"]
    for i in range(n_modules):
        dom = _DOMAINS[i % len(_DOMAINS)] + ("" if i < len(_DOMAINS) else str(i))
        D = _cap(dom)
        base = os.path.join(root, "src", dom)
        _write(os.path.join(base, "dto", f"create-{dom}.dto.ts"),
               f"export class Create{D}Dto {{\n  name: string;\n  amount?: number;\n}}\n")
        _write(os.path.join(base, f"{dom}.entity.ts"),
               f"export interface {D}Entity {{ id: string; name: string; }}\n"
               f"export const make{D} = (id: string, name: string): {D}Entity => ({{ id, name }});\n")
        verbs = rnd.sample(_VERBS, 3)
        svc = "\n".join(f"  async {v}(id: string, dto: Create{D}Dto): Promise<{D}Entity> {{\n"
                        f"    return make{D}(id, dto.name);\n  }}\n" for v in verbs)
        _write(os.path.join(base, f"{dom}.service.ts"),
               f"import {{ Injectable }} from '@nestjs/common';\nimport {{ Create{D}Dto }} from './dto/create-{dom}.dto';\n"
               f"import {{ {D}Entity, make{D} }} from './{dom}.entity';\n\n@Injectable()\nexport class {D}Service {{\n"
               f"  private readonly cache = new Map<string, {D}Entity>();\n\n{svc}\n"
               f"  findAll = async (): Promise<{D}Entity[]> => [...this.cache.values()];\n}}\n")
        routes = "\n".join(f"  @Post('{v}/:id')\n  {v}(@Param('id') id: string, @Body() dto: Create{D}Dto) {{\n"
                           f"    return this.service.{v}(id, dto);\n  }}\n" for v in verbs)
        _write(os.path.join(base, f"{dom}.controller.ts"),
               f"import {{ Body, Controller, Get, Param, Post }} from '@nestjs/common';\n"
               f"import {{ {D}Service }} from './{dom}.service';\nimport {{ Create{D}Dto }} from './dto/create-{dom}.dto';\n\n"
               f"@Controller('{dom}s')\nexport class {D}Controller {{\n  constructor(private readonly service: {D}Service) {{}}\n\n"
               f"  @Get()\n  findAll() {{\n    return this.service.findAll();\n  }}\n\n{routes}}}\n")
        idents += [f"{dom}.dto.create-{dom}.dto", f"{dom}.{dom}.entity", f"{dom}.{dom}.service",
                   f"{dom}.{dom}.controller"]
    if commit:
        _git_commit(root)
    return idents


def go_gin_repo(root: str, n_packages: int = 6, module: str = "github.com/acme/gosvc", commit: bool = True) -> List[str]:
    _write(os.path.join(root, "go.mod"), f"module {module}\n\ngo 1.22\n")
    _write(os.path.join(root, "cmd", "server", "main.go"),
           f'package main\n\nimport (\n\t"github.com/gin-gonic/gin"\n\t"{module}/internal/handler"\n)\n\n'
           "func main() {\n\tr := gin.Default()\n\thandler.Register(r)\n\t_ = r.Run()\n}\n")
    pkgs = [f"{module}/cmd/server"]
    regs = []
    for i in range(n_packages):
        dom = _DOMAINS[i % len(_DOMAINS)]
        D = _cap(dom)
        _write(os.path.join(root, "internal", "model", f"{dom}.go"),
               f"package model\n\n// {D} is a domain record.\ntype {D} struct {{\n\tID   string `json:\"id\"`\n\tName string\n}}\n")
        _write(os.path.join(root, "internal", f"{dom}service", "service.go"),
               f'package {dom}service\n\nimport (\n\t"context"\n\t"errors"\n\n\t"{module}/internal/model"\n)\n\n'
               f"// Service implements {dom} rules.\ntype Service struct{{ items map[string]*model.{D} }}\n\n"
               f"// Get loads one {dom}.\nfunc (s *Service) Get(ctx context.Context, id string) (*model.{D}, error) {{\n"
               f"\tif s.items == nil {{\n\t\tpanic(\"uninitialized\")\n\t}}\n\tv, ok := s.items[id]\n"
               f"\tif !ok {{\n\t\treturn nil, errors.New(\"not found\")\n\t}}\n\treturn v, nil\n}}\n\n"
               f"// Save stores a {dom}.\nfunc (s *Service) Save(ctx context.Context, v *model.{D}) error {{\n"
               f"\ts.items[v.ID] = v\n\treturn nil\n}}\n")
        pkgs.append(f"{module}/internal/{dom}service")
        regs.append(dom)
    pkgs.append(f"{module}/internal/model")
    imports = "\n".join(f'\t"{module}/internal/{d}service"' for d in regs)
    handlers = "\n".join(f"func {_cap(d)}Get(c *gin.Context) {{\n\tvar s {d}service.Service\n\t_, _ = s.Get(c, c.Param(\"id\"))\n}}\n"
                         for d in regs)
    routes = "\n".join(f'\tr.GET("/{d}/:id", {_cap(d)}Get)' for d in regs)
    _write(os.path.join(root, "internal", "handler", "routes.go"),
           f'package handler\n\nimport (\n\t"github.com/gin-gonic/gin"\n{imports}\n)\n\n{handlers}\n'
           f"// Register wires the HTTP routes.\nfunc Register(r *gin.Engine) {{\n{routes}\n}}\n")
    pkgs.append(f"{module}/internal/handler")
    if commit:
        _git_commit(root)
    return pkgs


def go_service_repo(root: str, n_packages: int = 250, module: str = "github.com/acme/gomono",
                    commit: bool = True) -> List[str]:
    """A large Go service (bench.py extra.goIndex, BASELINE config 5 at scale):
    ``n_packages`` domain packages of 4 files each (types, repository,
    service with a panic path, gin handlers) + cmd/server, every package
    name unique, handlers registered from main."""
    _write(os.path.join(root, "go.mod"), f"module {module}\n\ngo 1.22\n")
    pkgs = []
    names = []
    for i in range(n_packages):
        dom = _DOMAINS[i % len(_DOMAINS)] + str(i // len(_DOMAINS))
        D = _cap(dom)
        base = os.path.join(root, "internal", dom)
        _write(os.path.join(base, "types.go"),
               f"package {dom}\n\n// {D} is a domain record.\ntype {D} struct {{\n\tID   string `json:\"id\"`\n"
               f"\tName string\n\tAmount int64\n}}\n\n// Store persists {dom} records.\ntype Store interface {{\n"
               f"\tLoad(id string) (*{D}, error)\n\tSave(v *{D}) error\n}}\n")
        _write(os.path.join(base, "repository.go"),
               f'package {dom}\n\nimport "errors"\n\n// MemStore keeps {dom} records in memory.\n'
               f"type MemStore struct{{ items map[string]*{D} }}\n\n"
               f"// Load returns one record.\nfunc (m *MemStore) Load(id string) (*{D}, error) {{\n"
               f"\tv, ok := m.items[id]\n\tif !ok {{\n\t\treturn nil, errors.New(\"not found\")\n\t}}\n\treturn v, nil\n}}\n\n"
               f"// Save stores one record.\nfunc (m *MemStore) Save(v *{D}) error {{\n\tm.items[v.ID] = v\n\treturn nil\n}}\n")
        dep = _DOMAINS[(i + 1) % len(_DOMAINS)] + str(((i + 1) % n_packages) // len(_DOMAINS))
        imp = f'\n\t"{module}/internal/{dep}"' if i + 1 < n_packages else ""
        use = f"\n\tvar _ *{dep}.{_cap(dep)}" if i + 1 < n_packages else ""
        _write(os.path.join(base, "service.go"),
               f'package {dom}\n\nimport (\n\t"context"{imp}\n)\n\n// Service implements the {dom} rules.\n'
               f"type Service struct{{ store Store }}\n\n"
               f"// Get loads one {dom}.\nfunc (s *Service) Get(ctx context.Context, id string) (*{D}, error) {{\n"
               f"\tif s.store == nil {{\n\t\tpanic(\"uninitialized\")\n\t}}{use}\n\treturn s.store.Load(id)\n}}\n\n"
               f"// Update changes the amount of a {dom}.\nfunc (s *Service) Update(ctx context.Context, id string, amount int64) error {{\n"
               f"\tv, err := s.Get(ctx, id)\n\tif err != nil {{\n\t\treturn err\n\t}}\n\tv.Amount = amount\n"
               f"\treturn s.store.Save(v)\n}}\n")
        _write(os.path.join(base, "handler.go"),
               f'package {dom}\n\nimport "github.com/gin-gonic/gin"\n\n// Handler serves {dom} over HTTP.\n'
               f"type Handler struct{{ svc *Service }}\n\n// Get handles GET /{dom}/:id.\n"
               f"func (h *Handler) Get(c *gin.Context) {{\n\t_, _ = h.svc.Get(c, c.Param(\"id\"))\n}}\n\n"
               f"// Register wires the routes.\nfunc Register(r *gin.Engine, h *Handler) {{\n"
               f'\tr.GET("/{dom}/:id", h.Get)\n}}\n')
        pkgs.append(f"{module}/internal/{dom}")
        names.append(dom)
    imports = "\n".join(f'\t"{module}/internal/{d}"' for d in names[:50])
    regs = "\n".join(f"\t{d}.Register(r, &{d}.Handler{{}})" for d in names[:50])
    _write(os.path.join(root, "cmd", "server", "main.go"),
           f'package main\n\nimport (\n\t"github.com/gin-gonic/gin"\n{imports}\n)\n\n'
           f"func main() {{\n\tr := gin.Default()\n{regs}\n\t_ = r.Run()\n}}\n")
    pkgs.append(f"{module}/cmd/server")
    if commit:
        _git_commit(root)
    return pkgs


def stack_trace_for(fqcns: List[str], frames: int = 20, seed: int = 11) -> List[dict]:
    """A plausible 20-frame Java stack trace over a synthetic repo."""
    rnd = random.Random(seed)
    ctrls = [f for f in fqcns if f.endswith("Controller")]
    svcs = [f for f in fqcns if f.endswith("Service")]
    repos = [f for f in fqcns if f.endswith("Repository")]
    out = []
    for i in range(frames):
        pool = [ctrls, svcs, repos][i % 3] or fqcns
        cls = rnd.choice(pool)
        method = {"Controller": "list", "Service": "list", "Repository": "findAll"}.get(
            next((k for k in ("Controller", "Service", "Repository") if cls.endswith(k)), ""), "run")
        out.append({"className": cls, "methodName": method, "lineNumber": 10 + i})
    out.append({"className": "org.springframework.web.servlet.DispatcherServlet", "methodName": "doDispatch",
                "lineNumber": 1067})
    return out[:frames]


def llama_checkpoint(root: str, layers: int = 16, hidden: int = 2048, heads: int = 32, kv_heads: int = 8,
                     intermediate: int = 8192, vocab: int = 128256, tokenizer: str = "code-bpe-128k",
                     outliers=(7, 300, 1029, 1800), seed: int = 11, device: str = "cuda") -> str:
    """A Llama-format checkpoint directory (``config.json``, one
    ``model.safetensors``, ``tokenizer.json``) with *trained-like* random
    weights -- no download exists here: heavy-tailed matrices (a Gaussian
    scale mixture with log-normal scales), RMSNorm weights around 1 with a
    spread, and a few residual channels (``outliers``) carried at ~100x the
    others and damped by small norm weights, as trained Llama checkpoints
    show.  Llama-3.2-1B geometry by default (2.5 GB), the shipped 128,256-id
    code BPE as its tokenizer.  The tensors are drawn on ``device``."""
    import gzip
    import json

    import torch
    from safetensors.torch import save_file
    os.makedirs(root, exist_ok=True)
    g = torch.Generator(device=device).manual_seed(seed)
    hd = hidden // heads
    out = [o for o in outliers if o < hidden]

    def heavy(shape, std):
        x = torch.randn(shape, generator=g, device=device)
        x *= torch.exp(0.6 * torch.randn(shape, generator=g, device=device))
        return (x * (std / 1.2)).to(torch.bfloat16).cpu()

    def norm_w():
        w = 1.0 + 0.25 * torch.randn(hidden, generator=g, device=device)
        w[out] = 0.01
        return w.to(torch.bfloat16).cpu()
    emb = torch.randn(vocab, hidden, generator=g, device=device) * 0.02
    emb[:, out] *= 100.0
    t = {"model.embed_tokens.weight": emb.to(torch.bfloat16).cpu(), "lm_head.weight": heavy((vocab, hidden), 0.02),
         "model.norm.weight": norm_w()}
    del emb
    out_std = 0.02 / (2 * layers) ** 0.5
    for i in range(layers):
        p = f"model.layers.{i}."
        t[p + "input_layernorm.weight"] = norm_w()
        t[p + "post_attention_layernorm.weight"] = norm_w()
        t[p + "self_attn.q_proj.weight"] = heavy((heads * hd, hidden), 0.02)
        t[p + "self_attn.k_proj.weight"] = heavy((kv_heads * hd, hidden), 0.02)
        t[p + "self_attn.v_proj.weight"] = heavy((kv_heads * hd, hidden), 0.02)
        t[p + "self_attn.o_proj.weight"] = heavy((hidden, heads * hd), out_std)
        t[p + "mlp.gate_proj.weight"] = heavy((intermediate, hidden), 0.02)
        t[p + "mlp.up_proj.weight"] = heavy((intermediate, hidden), 0.02)
        t[p + "mlp.down_proj.weight"] = heavy((hidden, intermediate), out_std)
    save_file(t, os.path.join(root, "model.safetensors"))
    del t
    cfg = {"vocab_size": vocab, "hidden_size": hidden, "num_hidden_layers": layers, "num_attention_heads": heads,
           "num_key_value_heads": kv_heads, "intermediate_size": intermediate, "rms_norm_eps": 1e-5,
           "rope_theta": 500000.0, "architectures": ["LlamaForCausalLM"]}
    if tokenizer:
        assets = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "models", "assets",
                              tokenizer)
        with gzip.open(os.path.join(assets, "tokenizer.json.gz"), "rb") as f, \
                open(os.path.join(root, "tokenizer.json"), "wb") as o:
            o.write(f.read())
        with open(os.path.join(assets, "tokenizer_meta.json")) as f:
            meta = json.load(f)
        cfg["bos_token_id"], cfg["eos_token_id"] = meta.get("bos_token_id"), meta.get("eos_token_id")
    with open(os.path.join(root, "config.json"), "w") as f:
        json.dump(cfg, f)
    return root
