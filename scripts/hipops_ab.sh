#!/usr/bin/env bash
# Builds the kernel library of git revision $1 (default HEAD) into
# dmcp/ops/ab/_hipops_<rev>.so (git-ignored), for an A/B against the working tree via
# DMCP_HIPOPS_SO (CPU host; the .so travels with the gpurun snapshot).
set -eu
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
D=build/ab/src_$REV
mkdir -p dmcp/ops/ab
rm -rf "$D" && mkdir -p "$D"
for f in $(git ls-tree --name-only "$REV" dmcp/ops/csrc/); do git show "$REV:$f" > "$D/$(basename "$f")"; done
python3 - "$D" "dmcp/ops/ab/_hipops_$REV.so" <<'PY'
import subprocess, sys, glob
from dmcp.ops import build as b
srcs = sorted(glob.glob(sys.argv[1] + "/*.hip"))
subprocess.run([b.hipcc(), *b.FLAGS, "-shared", f"-I{sys.argv[1]}", "-o", sys.argv[2], *srcs], check=True)
print(sys.argv[2])
PY
