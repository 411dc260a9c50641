#!/bin/bash
# Round 4: the host enqueue probe alone (archive/tools_exp/enqueue_probe.py, 20 frames, 30 reps)
set -o pipefail
timeout -k 10 300 python3 archive/tools_exp/enqueue_probe.py 20 30 || exit 1
