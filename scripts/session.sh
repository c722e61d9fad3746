#!/bin/bash
# One GPU-box session, parameterised by the steps to run, in order (replaces the one-off
# scripts/gpu_r0x*.sh of rounds 3-4).  Every GPU step has its own time limit; the first
# failing step ends the session (no retries).  Outputs go to gpurun_out/TAG/.
#
#   bash scripts/session.sh TAG STEP [STEP ...]
#
# STEP is one of
#   smoke                      __graft_entry__.smoke()
#   tests[:K_EXPR]             pytest -m gpu (optionally -k K_EXPR)
#   testsall                   pytest -m gpu without -x (every failure in one run)
#   bench                      the headline bench line (bench.json)
#   prof                       rocprofv3 --kernel-trace --stats: headline alone, then every side line
#   pmc                        PMC traffic passes of the headline (scripts/gpu_profile.sh)
#   ab:SCRIPT:VARIANTS:REPS[:K=V,K=V]
#                              run python3 SCRIPT for each build in VARIANTS (comma-separated;
#                              "default" = lib/libtgms.so, else lib/variants/libtgms_NAME.so),
#                              alternating, REPS rounds, extra environment K=V; one JSON line
#                              per run (prefixed with the variant) into ab_SCRIPT.jsonl
#   vtests:VARIANT[:K_EXPR]    pytest -m gpu on a variant build
#   pmcs:SCRIPT:VARIANT:SETS[:K=V,K=V]
#                              rocprofv3 --pmc passes (one counter group per run, --kernel-trace
#                              only) of python3 SCRIPT on one build; SETS is a '+'-joined list of
#                              occ, inst, lds, fp64, bytes; per-kernel means folded by
#                              scripts/pmc_fold.py into pmc_SCRIPT_VARIANT.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
V=trajectory_generator_ros2_amd/lib/variants
SIDE_OFF="--dense-steps 0 --band-steps 0 --sample-traj 0 --config5 0 --config4 0 --cache-resident 0 --host-line 0 --node-line 0 --uniform-large-m 0 --config2 0"

declare -A PMC_SETS=(
    [occ]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
    [inst]="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
    [lds]="SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"
    [fp64]="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES"
    [bytes]="FETCH_SIZE|WRITE_SIZE"
)
end() { echo "step '$1' failed (rc $2): session ends"; exit "$2"; }
libpath() { if [ "$1" = default ]; then echo ""; else echo "$V/libtgms_$1.so"; fi; }
pytest_gpu() {  # LOG [K_EXPR]
    if [ -n "${2:-}" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$2" > "$1" 2>&1
    else
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$1" 2>&1
    fi
}

for step in "$@"; do
    IFS=: read -r kind a b c d <<< "$step"
    echo "== $step"
    case $kind in
    smoke)
        timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || end "$step" $?
        tail -1 "$OUT/smoke.log" ;;
    tests)
        log="$OUT/pytest_gpu${a:+_$(echo "$a" | tr -c 'a-zA-Z0-9_\n' '_')}.log"
        pytest_gpu "$log" "${a:-}"; rc=$?
        tail -3 "$log"
        [ $rc -eq 0 ] || end "$step" $rc ;;
    testsall)
        timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
            > "$OUT/pytest_gpu_all.log" 2>&1; rc=$?
        tail -15 "$OUT/pytest_gpu_all.log"
        [ $rc -eq 0 ] || end "$step" $rc ;;
    vtests)
        log="$OUT/pytest_gpu_$a.log"
        TGMS_LIB=$(libpath "$a") pytest_gpu "$log" "${b:-}"; rc=$?
        tail -3 "$log"
        [ $rc -eq 0 ] || end "$step" $rc ;;
    bench)
        timeout -k 10 300 python bench.py --steps 50 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || end "$step" $?
        cut -c1-400 "$OUT/bench.json" ;;
    prof)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
            python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 $SIDE_OFF > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || end "$step" $?
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_full" -o run --output-format csv -- \
            python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --dense-steps 2 > "$OUT/prof_full_bench.json" 2> "$OUT/prof_full.err" || end "$step" $?
        find "$OUT/prof" "$OUT/prof_full" -name '*stats*' ;;
    pmc)
        bash scripts/gpu_profile.sh || end "$step" $?
        cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json" ;;
    ab)
        script=$a; variants=$b; reps=${c:-3}; envs=${d:-}
        name=$(basename "$script" .py)
        for r in $(seq 1 "$reps"); do
            for v in ${variants//,/ }; do
                line=$(env ${envs//,/ } TGMS_LIB=$(libpath "$v") timeout -k 10 300 python3 "$script" 2>> "$OUT/ab_$name.err") || end "$step" $?
                echo "{\"variant\": \"$v\", \"rep\": $r, \"env\": \"$envs\", \"out\": $line}" >> "$OUT/ab_$name.jsonl"
            done
        done
        cut -c1-260 "$OUT/ab_$name.jsonl" | tail -n $(( reps * $(echo "$variants" | tr ',' '\n' | wc -l) )) ;;
    pmcs)
        script=$a; v=$b; sets=$c; envs=${d:-}
        tag="$(basename "$script" .py)_$v"
        mkdir -p "$OUT/pmc_$tag"
        i=0
        for set in ${sets//+/ }; do
            IFS='|' read -ra groups <<< "${PMC_SETS[$set]}"
            for grp in "${groups[@]}"; do
                i=$((i + 1))
                env ${envs//,/ } TGMS_LIB=$(libpath "$v") timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace \
                    --output-format csv -d "$OUT/pmc_$tag/p$i" -o run -- python3 "$script" \
                    > "$OUT/pmc_$tag/p$i.json" 2> "$OUT/pmc_$tag.p$i.err" || end "$step ($grp)" $?
            done
        done
        python3 scripts/pmc_fold.py "$OUT/pmc_$tag" > "$OUT/pmc_$tag.txt" || end "$step (fold)" $?
        cat "$OUT/pmc_$tag.txt" ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
echo "session $TAG done"
