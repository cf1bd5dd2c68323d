#!/bin/bash
# round 6 session ah: the round's build -- every GPU test, smoke, the default
# bench line, the headline's kernel trace and PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_session.sh r06ah tests smoke bench trace pmc
