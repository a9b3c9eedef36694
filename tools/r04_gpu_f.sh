#!/bin/bash
# round 4: team exchange sweeps issue every granule load before testing -- suite, probes, small-K A/B
set -o pipefail
bash tools/r04_team_ab.sh || exit 1
bash tools/r04_team_xchg.sh || exit 1
