# Round-5 stall counters: per-kernel instruction mix, LDS conflicts and wait fractions of the bf16
# 64^3 B=4 step (three 8-counter SQ passes over eager bench steps) + the plan-mode kernel trace.
# Every step under its own time limit; a kill or timeout ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5stall
cd /tmp && export TMPDIR=/tmp
rm -rf $O && mkdir -p $O
chk() { rc=$1; if [ $rc -ge 124 ]; then echo "step rc=$rc, stopping"; exit $rc; fi; }
B64="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --mode eager"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -o run -- python3 $B64 > $O/p1.log 2>&1; chk $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $B64 > $O/p2.log 2>&1; chk $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sub > $O/trace.json 2> $O/trace.err; chk $?
python3 $R/tools/pmc_r5_summary.py stall $O/p1 $O/p2 $O/trace --json $O/stalls.json > $O/stalls.txt; chk $?
echo done
