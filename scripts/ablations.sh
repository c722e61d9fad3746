#!/bin/bash
# Ablation builds of the lane kernel (config 3), built here, timed on the GPU box:
#   bash scripts/ablations.sh && gpurun -- 'bash scripts/session.sh abl ab:scripts/kbench.py:default,nostore,nsns,noemit,nsne:3'
# nostore: no coefficient stores; nsns: no stores and no LDS staging; noemit: no
# coefficient arithmetic (stores kept); nsne: neither stores nor coefficient arithmetic.
set -e
cd "$(dirname "$0")/.."
python3 scripts/build_variant.py nostore tgms_reduced.hip -DTGMS_ABL_NOSTORE
python3 scripts/build_variant.py nsns tgms_reduced.hip -DTGMS_ABL_NOSTORE -DTGMS_ABL_NOSTAGE
python3 scripts/build_variant.py noemit tgms_reduced.hip -DTGMS_ABL_NOEMIT
python3 scripts/build_variant.py nsne tgms_reduced.hip -DTGMS_ABL_NOSTORE -DTGMS_ABL_NOEMIT
