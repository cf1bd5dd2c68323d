#!/bin/bash
# round 6 session ac: sessions z (per-packet, this build against the last
# commit's library), ab (tools/dispatch_probe) and aa (kernarg placement
# settings against the headline step) in one call
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/sessions/gpu_r06ab.sh && bash tools/sessions/gpu_r06z.sh && bash tools/sessions/gpu_r06aa.sh
