"""Process / device parallelism.

* :mod:`.dist` -- one-process-per-GPU ``torch.distributed`` plumbing (RCCL on
  ROCm, gloo on CPU): rank discovery, barriers, MAX/SUM reductions, used by
  the benchmarks;
* :mod:`.replicas` -- data-parallel pool of local-LLM engines (one replica per
  GPU, work-stealing over classes; no collectives in the hot path);
* :mod:`.bulk` -- bulk repository indexing across worker processes (the
  reference's sequential ``scripts/analyze-repos.sh``).
"""
