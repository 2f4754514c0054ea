# gpu_steps.sh -- the GPU-box measurement steps, one script (developer tool; the steps DESIGN.md cites).
#
# usage (from the repo root, on the GPU box):  TAG=name bash java-rsync_amd/tools/gpu_steps.sh STEP [STEP ...]
# Outputs go to gpurun_out/$TAG/.  Every step runs under its own time limit; the first step that fails (a test
# failure, a fault, an abort or a time limit) ends the call, so nothing else touches the GPU after it.
#
#   tests        the whole GPU suite (pytest -m gpu)
#   tests-batch  the batched-scan suite and the config-4 oracle checks
#   pytest       the GPU tests named in PYTEST_ARGS (files / -k expressions)
#   smoke        __graft_entry__.smoke()
#   bench        the default bench line (config 5, with companions)
#   files        the config-4 line, both basis forms (FILES_STEPS steps)
#   files-trace  one traced config-4 step (VARIANT, default half; FT_ARGS: more bench args): the chain walk's breakdown
#   prof         rocprofv3 kernel trace + stats of the default line (the summary committed under profiles/)
#   timeline     rocprofv3 kernel + copy timeline of the config-4 line (VARIANT; TL_ARGS: more bench args)
#   hl           the config-5 headline alone (no companions, no config 4), 20 steps
#   hl-trace     rocprofv3 kernel + copy trace of the headline alone, and its per-step gaps (tools/step_gaps.py)
#   fetch        rocprofv3 --pmc FETCH_SIZE passes (counters only, kernel trace) of the default line and the config-4
#                line: the HBM bytes per K1 launch that bench.py reports as roofline.traffic
#   pmc-k1       one PMC pass over kbench: the production K1 against the same kernel without global loads
#   pmc-walk     two PMC passes (SQ issue/wait/LDS counters) over one config-4 step (VARIANT; PMC_ARGS: more bench
#                args): the chain walk's instruction mix and LDS bank conflicts
#   kbench-k1    kbench: the K1 at B = 128 KiB and 8 KiB, the batched forms (1002, 1005)
#   e2e          java-rsync_amd/tools/e2e.py at config 5 (16 GiB from host memory)
#   kb-ab        kbench A/Bs of KB_VARIANTS (default: the production entries 1000 1001 1003) at the headline
#                shape, interleaved, then one clock pass (GRBM_GUI_ACTIVE) over the same variants
#   kb-gather    kbench's Receiver block-gather A/Bs (KBENCH_GATHER: 4 GiB as 1 MiB ops)
#   e2e4         java-rsync_amd/tools/e2e_config4.py: config 4's shard (128 x 128 MiB) from host memory, the segment
#                entry points against 128 single-file calls
#   config3      the config-3 line: a 64 GiB identical pair resident in HBM, B = 131072 (the Sender's limit), dl = 5
#   receiver     the Receiver line (combineDataToFile on the config-2 shape)
#   multi        bench.py --gpus 2 without a launcher (its own rank processes) on a one-GPU box: the N-rank path,
#                ranks sharing the GPU (a rehearsal, not a scaling point); config 5 and config 4
#   devices      bench.py --workload files --devices N in one process (rsh_*_batch_multi from host memory): the same 128
#                files over 1 context and over 2 (both on GPU 0 on a one-GPU box: the plumbing, not a scaling point)
#   first        tools/first_call.py: the first calls on a fresh context against the later ones (config 4, config 5)
#   first4       first_call.py --only 4 with --trim: the config-4 segment scan's first calls, device-resident (traced) and
#                from host memory, and a segment after rsh_ctx_trim
#   first-trace  rocprofv3 HIP API + kernel trace of first_call.py --only 5 --reps 2 (where the first step's time goes)
#   copycb       rocprofv3 --memory-copy-trace over tools/queue_lat.hip (3 D2H hipMemcpyAsync per rep, no librsynchip):
#                does the profiler report undelivered copy completions for plain runtime copies too
#   copycb5      rocprofv3 --memory-copy-trace --hip-trace over first_call.py --only 5 (then --only 4): which of the
#                library's copies the profiler reports undelivered
#   copycb-files the same over the config-4 line (VARIANT): which copies of the timeline run stay undelivered
#   libab        builds of other commits against each other (LIBS: directories under java-rsync_amd/lib/ab, each holding a
#                librsynchip.so, loaded through RSH_LIB), alternating, REPS times (AB_ARGS: bench args)
#   ab           AB_OPTS ("name=value ...") against the default, alternating, REPS times (AB_ARGS: bench args; AB_LIB:
#                the library both arms load, default the diagnostics build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-steps}
mkdir -p "$O"
cd "$R"
K=$R/java-rsync_amd/lib/kbench
VARIANT=${VARIANT:-half}

run() {  # run LIMIT cmd... : the step's own time limit; any failure ends the call
    local lim=$1
    shift
    timeout -k 10 "$lim" "$@" || { echo "step failed ($?): $*"; exit 1; }
}

for step in "$@"; do
    echo "[gpu_steps] $step"
    case $step in
        tests) run 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$O/gpu_tests.log" 2>&1 ;;
        tests-batch) run 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_batch.py \
            tests/test_gpu_fullsize.py -k "batch or config4" > "$O/batch_tests.log" 2>&1 ;;
        pytest) run 900 python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread $PYTEST_ARGS \
            > "$O/pytest.log" 2>&1 ;;
        kb-ab)
            V=${KB_VARIANTS:-"1000 1001 1003"}
            run 240 "$K" 16384 131072 4 6 $V $V $V > "$O/kb_ab.log" 2>&1
            (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace \
                -d "$O/kb_ab_clock" -o run --output-format csv -- "$K" 16384 131072 4 5 $V > "$O/kb_ab_clock.log" 2>&1) \
                || exit 1
            python3 java-rsync_amd/tools/clock_summary.py "$O/kb_ab_clock" > "$O/kb_ab_clock.txt" 2>&1 ;;
        kb-gather) KBENCH_GATHER=1048576 run 180 "$K" 4096 0 0 5 0 1 2 3 4 5 6 0 1 2 3 4 5 6 > "$O/kb_gather.log" 2>&1 ;;
        e2e4) run 900 python java-rsync_amd/tools/e2e_config4.py $E2E4_ARGS > "$O/e2e_config4.json" 2> "$O/e2e_config4.err" ;;
        smoke) run 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 ;;
        bench) run 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" ;;
        hl) run 240 python bench.py --no-companions --no-files --no-cpu-baseline --steps 20 --warmup 5 $HL_ARGS \
            > "$O/hl.json" 2> "$O/hl.err" ;;
        hl-trace) (cd /tmp && export TMPDIR=/tmp && run 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/hl_trace" \
            -o run --output-format csv -- python3 "$R/bench.py" --no-companions --no-files --no-cpu-baseline --steps 10 \
            --warmup 3 $HL_ARGS > "$O/hl_trace.json" 2> "$O/hl_trace.err") || exit 1
            python3 java-rsync_amd/tools/step_gaps.py "$O/hl_trace" > "$O/hl_gaps.txt" 2>&1 ;;
        files)
            for v in half identical; do
                run 300 python bench.py --workload files --variant $v --steps "${FILES_STEPS:-8}" --warmup 2 \
                    --no-cpu-baseline --no-companions > "$O/files_$v.json" 2> "$O/files_$v.err"
            done ;;
        files-trace) run 300 python bench.py --workload files --variant "$VARIANT" --steps 1 --warmup 1 --no-cpu-baseline \
            --no-companions --opt scan_trace=2 $FT_ARGS > "$O/files_${VARIANT}_trace.json" 2> "$O/files_${VARIANT}_trace.err" ;;
        prof) (cd /tmp && export TMPDIR=/tmp && run 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run \
            --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline \
            > "$O/prof_bench.json" 2> "$O/prof_bench.err") || exit 1 ;;
        timeline) (cd /tmp && export TMPDIR=/tmp && run 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
            -d "$O/timeline" -o run --output-format csv -- python3 "$R/bench.py" --workload files --variant "$VARIANT" \
            --steps 3 --warmup 1 --no-cpu-baseline --no-companions $TL_ARGS > "$O/timeline.json" 2> "$O/timeline.err") || exit 1 ;;
        fetch)
            (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o run \
                --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-companions \
                > "$O/fetch_bench.json" 2> "$O/fetch_bench.err") || exit 1
            (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch_files" -o run \
                --output-format csv -- python3 "$R/bench.py" --workload files --steps 2 --warmup 1 --no-cpu-baseline \
                --no-companions > "$O/fetch_files.json" 2> "$O/fetch_files.err") || exit 1 ;;
        pmc-k1)
            C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
            run 120 "$K" 16384 131072 4 5 1000 58 > "$O/pmc_kbench.log" 2>&1
            (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d "$O/pmc" -o run \
                --output-format csv -- "$K" 16384 131072 4 3 1000 58 > "$O/pmc.log" 2>&1) || exit 1 ;;
        pmc-walk)
            # two PMC passes over one config-4 step (every kernel; the chain walk is chain_advance_kernel)
            CA="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
            CB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
            (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $CA --kernel-trace -d "$O/pmc_walk_a" -o run \
                --output-format csv -- python3 "$R/bench.py" --workload files --variant "$VARIANT" --steps 1 --warmup 1 \
                --no-cpu-baseline --no-companions $PMC_ARGS > "$O/pmc_walk_a.json" 2> "$O/pmc_walk_a.err") || exit 1
            (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $CB --kernel-trace -d "$O/pmc_walk_b" -o run \
                --output-format csv -- python3 "$R/bench.py" --workload files --variant "$VARIANT" --steps 1 --warmup 1 \
                --no-cpu-baseline --no-companions $PMC_ARGS > "$O/pmc_walk_b.json" 2> "$O/pmc_walk_b.err") || exit 1 ;;
        k1-energy)  # the production K1 (1000) against its VALU weak-sum form (1010), interleaved; then one PMC pass
            run 180 "$K" 16384 131072 4 5 1000 1010 1000 1010 > "$O/k1_energy_kbench.log" 2>&1
            C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
            (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d "$O/k1_energy_pmc" -o run \
                --output-format csv -- "$K" 16384 131072 4 3 1000 1010 1000 1010 > "$O/k1_energy_pmc.log" 2>&1) || exit 1 ;;
        kbench-k1)
            run 120 "$K" 16384 131072 4 8 1000 > "$O/kbench_128k.log" 2>&1
            run 120 "$K" 16384 8192 3 8 1000 1002 1005 > "$O/kbench_8k.log" 2>&1 ;;
        multi)
            run 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-companions \
                > "$O/multi_file.json" 2> "$O/multi_file.err"
            run 300 python bench.py --gpus 2 --workload files --steps 5 --warmup 2 --no-cpu-baseline --no-companions \
                > "$O/multi_files.json" 2> "$O/multi_files.err" ;;
        devices)
            for d in 1 2; do
                run 400 python bench.py --workload files --variant "$VARIANT" --devices $d --files $((128 / d)) --steps 3 \
                    --warmup 1 > "$O/devices_$d.json" 2> "$O/devices_$d.err"
            done ;;
        config3) run 300 python bench.py --size-gib 64 --digest 5 --steps 3 --warmup 1 --no-companions --no-cpu-baseline \
            > "$O/config3.json" 2> "$O/config3.err" ;;
        receiver) run 300 python bench.py --workload receiver --steps 2 --warmup 1 > "$O/receiver.json" 2> "$O/receiver.err" ;;
        e2e) run 400 python java-rsync_amd/tools/e2e.py --gib 16 > "$O/e2e_16GiB.json" 2> "$O/e2e.err" ;;
        copycb) (cd /tmp && export TMPDIR=/tmp && run 120 rocprofv3 --memory-copy-trace --kernel-trace -d "$O/copycb" \
            -o run --output-format csv -- "$R/java-rsync_amd/lib/queue_lat" 4 > "$O/copycb.log" 2> "$O/copycb.err") || exit 1 ;;
        copycb5) for o in 5 4; do
                (cd /tmp && export TMPDIR=/tmp && run 240 rocprofv3 --memory-copy-trace --hip-trace -d "$O/copycb_$o" \
                    -o run --output-format csv -- python3 "$R/java-rsync_amd/tools/first_call.py" --only $o --reps 2 \
                    > "$O/copycb_$o.log" 2> "$O/copycb_$o.err") || exit 1
            done ;;
        copycb-files) (cd /tmp && export TMPDIR=/tmp && run 240 rocprofv3 --memory-copy-trace --hip-trace -d "$O/copycb_files" \
            -o run --output-format csv -- python3 "$R/bench.py" --workload files --variant "$VARIANT" --steps 3 --warmup 1 \
            --no-cpu-baseline --no-companions > "$O/copycb_files.json" 2> "$O/copycb_files.err") || exit 1 ;;
        libab)
            for r in $(seq 1 "${REPS:-2}"); do
                for l in $LIBS; do
                    RSH_LIB="$R/java-rsync_amd/lib/ab/$l/librsynchip.so" run 300 python bench.py $AB_ARGS --steps 20 \
                        --warmup 5 --no-cpu-baseline --no-companions > "$O/${l}_$r.json" 2> "$O/${l}_$r.err"
                done
            done ;;
        first) run 300 python java-rsync_amd/tools/first_call.py > "$O/first_call.json" 2> "$O/first_call.err" ;;
        first4) run 300 python java-rsync_amd/tools/first_call.py --only 4 --reps 4 --trim --trace $FIRST4_ARGS > "$O/first4.json" \
            2> "$O/first4.err"
            run 300 python java-rsync_amd/tools/first_call.py --only 4 --reps 3 --trim --host > "$O/first4_host.json" \
            2> "$O/first4_host.err" ;;
        first4-trace) (cd /tmp && export TMPDIR=/tmp && run 300 rocprofv3 --hip-trace --kernel-trace -d "$O/first4_trace" \
            -o run --output-format csv -- python3 "$R/java-rsync_amd/tools/first_call.py" --only 4 --reps 2 --trim \
            > "$O/first4_trace.json" 2> "$O/first4_trace.err") || exit 1 ;;
        first5) run 300 python java-rsync_amd/tools/first_call.py --only 5 --reps 4 --trace5 $FIRST5_ARGS > "$O/first5.json" \
            2> "$O/first5.err" ;;
        first-trace) (cd /tmp && export TMPDIR=/tmp && run 300 rocprofv3 --hip-trace --kernel-trace -d "$O/first_trace" \
            -o run --output-format csv -- python3 "$R/java-rsync_amd/tools/first_call.py" --only 5 --reps 2 \
            > "$O/first_trace.json" 2> "$O/first_trace.err") || exit 1 ;;
        ab)  # the A/B switches are settable in the diagnostics build only: both arms load it (AB_LIB: another build,
             # for product options)
            DIAG_LIB=${AB_LIB:-"$R/java-rsync_amd/lib/diag/librsynchip.so"}
            OPTS=""
            for o in $AB_OPTS; do OPTS="$OPTS --opt $o"; done
            for r in $(seq 1 "${REPS:-3}"); do
                RSH_LIB="$DIAG_LIB" run 300 python bench.py $AB_ARGS --steps 20 --warmup 5 --no-cpu-baseline --no-companions > "$O/a_$r.json" 2> "$O/a_$r.err"
                RSH_LIB="$DIAG_LIB" run 300 python bench.py $AB_ARGS --steps 20 --warmup 5 --no-cpu-baseline --no-companions $OPTS > "$O/b_$r.json" 2> "$O/b_$r.err"
            done ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
