#!/bin/bash
# Round 4, final build: the C4 profile set with the LW chain after the SW network (now the default there too).
set -u
export TMPDIR=/tmp
CONFIGS="c4" bash tools/profile_configs.sh
