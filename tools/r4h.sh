#!/bin/bash
# one call: VE_ACTIN checks + vocoder A/B, then the fused-FeedForward threshold A/B
bash tools/actin_check.sh || exit 1
bash tools/ffn_min_ab.sh
