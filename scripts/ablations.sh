#!/bin/bash
# Ablation builds of the lane kernel (config 3), built here, timed on the GPU box:
#   bash scripts/ablations.sh && gpurun -- 'bash scripts/gpu_kvar.sh nostore nsns noemit nsne'
# nostore: no coefficient stores; nsns: no stores and no LDS staging; noemit: no
# coefficient arithmetic (stores kept); nsne: neither stores nor coefficient arithmetic.
set -e
cd "$(dirname "$0")/.."
bash scripts/build_variant.sh nostore -DTGMS_ABL_NOSTORE
bash scripts/build_variant.sh nsns -DTGMS_ABL_NOSTORE -DTGMS_ABL_NOSTAGE
bash scripts/build_variant.sh noemit -DTGMS_ABL_NOEMIT
bash scripts/build_variant.sh nsne -DTGMS_ABL_NOSTORE -DTGMS_ABL_NOEMIT
