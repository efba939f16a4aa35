#!/bin/bash
# The vector-memory probes (not part of the product): per-
# instruction cost of byte / u64 rows and masked lanes (vmem_probe), page
# spread and masked-lane patterns (tlb_probe), Inflights ring layouts and
# partial stores (ring_probe).  Build them first on the host:
#   for p in vmem tlb ring; do hipcc -O3 --offload-arch=gfx950 -o scripts/${p}_probe scripts/${p}_probe.hip; done
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for p in vmem tlb ring; do
  timeout -k 10 120 ./scripts/${p}_probe > gpurun_out/${p}_probe.log 2>&1 || { echo "$p probe failed"; tail gpurun_out/${p}_probe.log; exit 3; }
  cat gpurun_out/${p}_probe.log
done
