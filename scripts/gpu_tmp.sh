set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sb gpurun_out/pmcB
timeout -k 10 120 ./scripts/storebench 65536 > gpurun_out/sb/sb65k.txt && timeout -k 10 120 ./scripts/storebench 524288 > gpurun_out/sb/sb512k.txt && cat gpurun_out/sb/*.txt || exit 1
for g in FETCH_SIZE WRITE_SIZE; do
  KB_B=524288 timeout -s KILL 90 rocprofv3 --pmc $g --kernel-trace --output-format csv -d gpurun_out/pmcB/$g -o run -- python3 scripts/kbench.py > gpurun_out/pmcB/$g.json 2>gpurun_out/pmcB/$g.err || exit 2
done
echo done
