#!/bin/bash
# Round 4, batch 3: step schedules (tools/r04_sched.sh), then the SW network occupancy variants and the 4-wave SW
# solver instance (tools/r04_mlpsw.sh).
set -u
bash tools/r04_sched.sh || exit $?
bash tools/r04_mlpsw.sh
