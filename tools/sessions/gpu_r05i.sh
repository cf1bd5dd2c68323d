#!/bin/bash
# round 5 session i: why the wide-slot golden case differs with the unsorted
# new-key path (VIGPATH_NK_CHECK: phase A's miss records against the host's
# CRC of their keys, both paths)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VIGPATH_NK_CHECK=1 timeout -k 10 200 python3 tools/sessions/r05i_dbg.py > gpurun_out/r05i_u.log 2>&1
grep -c "bad hashes 0 " gpurun_out/r05i_u.log; grep "nkcheck: seg" gpurun_out/r05i_u.log | grep -vc "bad hashes 0 "; grep "mismatches" gpurun_out/r05i_u.log
VIGPATH_NK_CHECK=1 VIGPATH_NK_SORTED=1 timeout -k 10 200 python3 tools/sessions/r05i_dbg.py > gpurun_out/r05i_s.log 2>&1
grep -c "bad hashes 0 " gpurun_out/r05i_s.log; grep "nkcheck: seg" gpurun_out/r05i_s.log | grep -vc "bad hashes 0 "; grep "mismatches" gpurun_out/r05i_s.log
grep -m12 "nkcheck: miss" gpurun_out/r05i_u.log
