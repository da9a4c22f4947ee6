# Round-5 counters: MFMA busy cycles of the bf16 64^3 step's kernels, and HBM bytes (FETCH_SIZE /
# WRITE_SIZE, separate passes) + a kernel trace of the 128^3 B=1 f32 step (BASELINE configs[2]).
# Every step under its own time limit; a kill or timeout ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5pmc
cd /tmp && export TMPDIR=/tmp
rm -rf $O && mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step rc=$rc, stopping"; exit $rc; fi; }
timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-sub > $O/bench.json 2> $O/bench.err; chk $?
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; chk $?
B64="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager"
B128="$R/bench.py --size 128 --batch 1 --precision f32 --no-cpu-baseline --no-sub"
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mfma -o run -- python3 $B64 > $O/mfma.log 2>&1; chk $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b64trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub > $O/b64trace.json 2> $O/b64trace.err; chk $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b128trace -o run -- python3 $B128 --steps 10 --warmup 2 > $O/b128trace.json 2> $O/b128trace.err; chk $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/b128fetch -o run -- python3 $B128 --steps 2 --warmup 1 --mode eager > $O/b128fetch.log 2>&1; chk $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/b128write -o run -- python3 $B128 --steps 2 --warmup 1 --mode eager > $O/b128write.log 2>&1; chk $?
echo done
