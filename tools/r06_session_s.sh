#!/bin/bash
# round-6 session s: final-tree profile -- GPU suite, default bench line, rocprofv3 kernel trace + stats
set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/round_profile.sh r06_v2
