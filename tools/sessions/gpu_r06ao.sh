#!/bin/bash
# round 6 session ao: the final tree -- every GPU test, smoke, the default
# bench line, the headline's kernel trace and PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r06ao tests smoke bench trace pmc
