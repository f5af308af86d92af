"""Process / device parallelism.

* :mod:`.dist` -- one-process-per-GPU ``torch.distributed`` plumbing (RCCL on
  ROCm, gloo on CPU): rank discovery, barriers, MAX/SUM reductions, used by
  the benchmarks;
* one local-LLM worker process per GPU lives in :mod:`dmcp.enrich.workers`
  (data-parallel over classes from one queue; no collectives in the hot path);
* :mod:`.bulk` -- bulk repository indexing across worker processes (the
  reference's sequential ``scripts/analyze-repos.sh``).
"""
