#!/bin/bash
# round 4: first GPU call = tools/gpu_r04_a.sh then tools/gpu_r04_b.sh
bash tools/gpu_r04_a.sh || exit $?
bash tools/gpu_r04_b.sh || exit $?
