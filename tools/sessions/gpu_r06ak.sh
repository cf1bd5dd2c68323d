#!/bin/bash
# round 6 session ak: the final tree -- every GPU test, smoke, the default
# bench line, and the N = 2 rehearsal (two ranks sharing the GPU, host
# transport) of the C-loop headline
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r06ak tests smoke bench shard2
