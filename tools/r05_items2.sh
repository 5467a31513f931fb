#!/bin/bash
# r05: the dense lookup's item count with the least-tail split (DFP_HJ_SLICED_ITEMS: 512 ->
# 2 parts per slice, 768 (default) -> 3, 1224 -> 4; the 50 slices past the whole rounds in
# fifths either way). tools/r05_env.sh A/B on C2 and C3.
RUNS="i768:DFP_HJ_SLICED_ITEMS=768 i512:DFP_HJ_SLICED_ITEMS=512 i1224:DFP_HJ_SLICED_ITEMS=1224" CFGS="c2 c3" BCFGS="c2 c3" REPS=2 bash tools/r05_env.sh ${1:-r05items2}
