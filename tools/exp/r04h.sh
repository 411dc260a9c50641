#!/bin/bash
set -o pipefail
timeout -k 10 300 python3 tools/exp/enqueue_probe.py 20 30 || exit 1
