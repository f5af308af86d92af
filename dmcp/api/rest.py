"""REST API (FastAPI) -- the reference's Spring MVC controllers.

Parity:

* ``POST /api/projects/analyze`` {repositoryUrl, branch?, fixMissed?=true}
  -> {success, projectId, classesAnalyzed, endpointsFound, message}; HTTP 500
  on failure (``AnalyzeProjectController.java:73-103``)
* ``POST /api/projects/{id}/rebuild-graph`` (``:126-148``)
* ``POST /api/projects/sync`` (``:171-196``)
* ``GET /api/projects`` -> {projects:[...]} without ``description``
  (``ProjectController.java:54-94``)
* ``GET /api/context/class/{className}``, ``GET /api/context/class?className=``,
  ``GET /api/context/method?className=&methodName=``,
  ``POST /api/context/stack-trace`` -- always 200 (``ContextController.java:62-153``)
* ``POST /api/graph/query`` {query} -> result, or 400 {error, errorCode}
  (``GraphQueryController.java:55-82``)
* ``GET /health`` -> ``up`` (``HealthController.java:19-22``)
* Swagger UI at ``/swagger-ui.html``, OpenAPI JSON at ``/api-docs``
  (``application.yml:62-68``)

Additions: ``POST /api/projects/{id}/resume-enrichment`` (checkpoint
resume), ``DELETE /api/projects/{id}`` (ProjectService.deleteProject, which
the reference never exposed), ``POST /api/tools/{name}`` (any MCP tool over
HTTP), ``GET /metrics`` (Prometheus text) and ``GET /api/stats``.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional

from fastapi import Body, FastAPI, HTTPException, Query
from fastapi.responses import JSONResponse, PlainTextResponse
from pydantic import BaseModel

from ..utils.errors import DomainError
from ..utils.tracing import METRICS
from .tools import ToolRegistry

LOG = logging.getLogger(__name__)


class AnalyzeRequest(BaseModel):
    repositoryUrl: str
    branch: Optional[str] = None
    fixMissed: Optional[bool] = None


class QueryRequest(BaseModel):
    query: Optional[str] = None


class StackFrameRequest(BaseModel):
    className: Optional[str] = None
    methodName: Optional[str] = None
    lineNumber: Optional[int] = None


class StackTraceRequest(BaseModel):
    stackTrace: List[StackFrameRequest] = []


DESCRIPTION = """Domain MCP Server - analyzes git repositories and serves their business
context to AI assistants.

* **Project analysis**: clone, statically parse (Java / TypeScript / Go), optionally enrich
* **Code context**: classes, methods, dependencies, service API
* **Stack trace correlation**: map Datadog frames to business meaning
* **Graph query DSL**: `project:target[:navigation]*[:+include]*[:?check]`
"""


def create_app(app) -> FastAPI:
    cfg = app.config
    api = FastAPI(title="Domain MCP Server API", version=cfg.mcp_server_version, description=DESCRIPTION,
                  openapi_url="/api-docs", docs_url="/swagger-ui.html", redoc_url=None,
                  servers=[{"url": cfg.app_url, "description": "API server"}])
    registry = ToolRegistry(app)

    @api.get("/health", response_class=PlainTextResponse, tags=["Health"])
    def health() -> str:
        return "up"

    # ------------------------------------------------------ project analysis
    @api.post("/api/projects/analyze", tags=["Project Analysis"])
    def analyze(req: AnalyzeRequest):
        fix = req.fixMissed is None or bool(req.fixMissed)
        try:
            r = app.indexer.analyze_project(req.repositoryUrl, req.branch, fix)
            return r.to_dict()
        except DomainError as e:
            LOG.error("Analysis failed: %s", e)
            return JSONResponse(status_code=500, content={"success": False, "projectId": None, "classesAnalyzed": 0,
                                                          "endpointsFound": 0, "message": e.message})
        except Exception as e:
            LOG.exception("Unexpected error during analysis")
            return JSONResponse(status_code=500, content={"success": False, "projectId": None, "classesAnalyzed": 0,
                                                          "endpointsFound": 0, "message": f"Internal error: {e}"})

    @api.post("/api/projects/{project_id}/rebuild-graph", tags=["Project Analysis"])
    def rebuild(project_id: str):
        try:
            app.indexer.rebuild_graph(project_id)
            return {"success": True, "projectId": project_id, "message": "Graph rebuilt successfully"}
        except DomainError as e:
            return JSONResponse(status_code=500, content={"success": False, "projectId": project_id,
                                                          "message": e.message})
        except Exception as e:
            return JSONResponse(status_code=500, content={"success": False, "projectId": project_id,
                                                          "message": f"Internal error: {e}"})

    @api.post("/api/projects/{project_id}/resume-enrichment", tags=["Project Analysis"])
    def resume(project_id: str):
        try:
            return app.indexer.resume_enrichment(project_id)
        except DomainError as e:
            return JSONResponse(status_code=500, content={"success": False, "projectId": project_id,
                                                          "message": e.message, "errorCode": e.error_code})

    @api.post("/api/projects/sync", tags=["Project Analysis"])
    def sync_all():
        r = app.indexer.sync_all_projects()
        return {"success": r.success, "totalProjects": r.total_projects, "successCount": r.success_count,
                "failureCount": r.failure_count,
                "projects": [{"projectName": x.project_name, "success": x.success, "addedClasses": x.added_classes,
                              "updatedClasses": x.updated_classes, "deletedClasses": x.deleted_classes,
                              "unchangedClasses": x.unchanged_classes, "errorMessage": x.error_message}
                             for x in r.results],
                "message": "Sync completed"}

    @api.delete("/api/projects/{project_id}", tags=["Project Analysis"])
    def delete_project(project_id: str):
        try:
            if not app.projects.delete_project(project_id):
                return JSONResponse(status_code=404, content={"success": False, "projectId": project_id,
                                                              "message": "Project not found"})
            return {"success": True, "projectId": project_id, "message": "Project deleted"}
        except DomainError as e:
            return JSONResponse(status_code=409, content={"success": False, "projectId": project_id,
                                                          "message": e.message, "errorCode": e.error_code})

    @api.get("/api/projects", tags=["Project Analysis"])
    def list_projects():
        out = []
        for p in app.context.list_projects():
            out.append({k: p[k] for k in ("id", "name", "repositoryUrl", "basePackage", "status",
                                          "lastAnalyzedAt", "classCount", "endpointCount")})
        return {"projects": out}

    # ----------------------------------------------------------- code context
    @api.get("/api/context/class/{class_name}", tags=["Code Context"])
    def class_context_path(class_name: str):
        return app.context.get_class_context(class_name)

    @api.get("/api/context/class", tags=["Code Context"])
    def class_context(className: str = Query(...)):
        return app.context.get_class_context(className)

    @api.get("/api/context/method", tags=["Code Context"])
    def method_context(className: str = Query(...), methodName: str = Query(...)):
        return app.context.get_method_context(className, methodName)

    @api.post("/api/context/stack-trace", tags=["Code Context"])
    def stack_trace(req: StackTraceRequest):
        frames = [f.model_dump() for f in req.stackTrace]
        return app.context.get_stack_trace_context(frames)

    # ------------------------------------------------------------ graph query
    @api.post("/api/graph/query", tags=["Graph Query"])
    def graph_query(req: QueryRequest):
        try:
            return app.graph_query.query(req.query).to_dict()
        except DomainError as e:
            return JSONResponse(status_code=400, content={"error": e.message, "errorCode": e.error_code})

    # ------------------------------------------------------------- extensions
    @api.post("/api/tools/{name}", tags=["MCP tools over HTTP"])
    def call_tool(name: str, arguments: Dict[str, Any] = Body(default={})):
        try:
            return registry.call(name, arguments)
        except KeyError:
            raise HTTPException(status_code=404, detail=f"Unknown tool: {name}")

    @api.get("/metrics", response_class=PlainTextResponse, tags=["Observability"])
    def metrics() -> str:
        return METRICS.prometheus()

    @api.get("/api/stats", tags=["Observability"])
    def stats():
        snap = METRICS.snapshot()
        snap["graphsCached"] = len(app.cache)
        return snap

    return api


def serve(app, host: Optional[str] = None, port: Optional[int] = None) -> None:
    import uvicorn
    api = create_app(app)
    app.start_scheduler()
    uvicorn.run(api, host=host or app.config.server_host, port=port or app.config.server_port,
                log_level=app.config.log_level.lower())
