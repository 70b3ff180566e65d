#!/bin/bash
# Parameterised GPU-box measurement steps (replaces the one-off rNNx.sh wrappers).
#   bash tools/steps.sh TAG STEP [STEP ...]
# Every step runs under its own time limit; the script stops at the first failing step (no retries).
# Output: gpurun_out/TAG/<step>.log (+ JSON lines of bench steps in <step>.json).
# Steps:
#   tests            the whole -m gpu suite
#   tests:<pattern>  pytest -m gpu -k <pattern>
#   mp               tests/test_gpu_multiprocess.py (rank processes over the IPC transport)
#   file:<path>      one GPU test file
#   smoke            __graft_entry__.smoke()
#   bench            default bench line (config 3, the driver's --steps 20 --warmup 5)
#   bench2           config 2 (one pmc_phase call per step)
#   slab1            config 3 through the slab driver, one rank, local halos
#   bench5box        the whole 256^3 / 8e7 box on one GPU
#   bench5           config 5 rehearsal (one 256x256x32 slab, halos through a one-rank RCCL communicator)
#   emu<R>[-<tp>][-d<us>][-ne|-t<k>]   config-4 rehearsal of R ranks (one rank's slab), transport tp (local|ipc|rccl,
#                    default local), injected exchange delay us, no events / events every k-th sweep
#   mp2bench         bench.py --gpus 2 --same-device --config 4 (rank processes, IPC); mp4bench, mp8bench: 4, 8
#   rocprof          rocprofv3 --kernel-trace --stats of the default bench command
#   trace8[d<us>]    rocprofv3 kernel trace of the 8-rank IPC rehearsal (injected exchange delay us) +
#                    tools/timeline_stats.py
#   py:<file>        python tools/<file> (analysis scripts, e.g. stamps.py with PMC_LIB_PATH=...@py:stamps.py)
#   tcc | sq | shcnt | slabtcc  counter passes: k_subsweep traffic (tools/tcc_traffic.sh), its SQ
#                    instruction mix (tools/sq_counters.sh), shiftCells traffic + wave states
#                    (tools/shift_counters.sh), the slab interior launches' traffic (tools/slab_traffic.sh)
# A step may carry environment variables: PMC_QUAD_CELLS=40000@bench2 (A/B switches).
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python -u -m pytest -x -q --timeout 180 --timeout-method thread"
summ() {   # one-line summary of a bench JSON line
    python3 - "$1" <<'EOF'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln); r = d.get("roofline") or {}; p = d.get("parity") or {}
        print("%s value %.4g ms/step %.4f issue %s launch %s phase %s shift %s frac %s parity %s/%s" % (
            sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"],
            "%.4f" % d["host_issue_ms_per_step"] if d.get("host_issue_ms_per_step") else None,
            "%.4f" % r["launch_ms"] if r.get("launch_ms") else None,
            "%.4f" % r["phase_ms"] if r.get("phase_ms") else None,
            "%.4f" % r["shift_ms"] if r.get("shift_ms") else None,
            "%.4f" % r["frac"] if r.get("frac") else None,
            p.get("state_bitwise_equal"), p.get("counters_equal")))
EOF
}
for spec in "$@"; do
    # VAR=VAL[,VAR=VAL...]@step runs the step with those environment variables (an A/B switch)
    envs=()
    step=$spec
    if [[ $spec == *@* ]]; then
        IFS=, read -ra envs <<< "${spec%%@*}"
        step=${spec#*@}
    fi
    name=${spec//[:\/=,@ ]/_}
    log=$OUT/$name.log
    echo "== $spec"
    for e in "${envs[@]}"; do export "$e"; done
    case $step in
        tests) timeout -k 10 900 $PYT tests -m gpu > $log 2>&1 ;;
        tests:*) timeout -k 10 600 $PYT tests -m gpu -k "${step#tests:}" > $log 2>&1 ;;
        mp) timeout -k 10 600 $PYT tests/test_gpu_multiprocess.py -m gpu > $log 2>&1 ;;
        file:*) timeout -k 10 700 $PYT ${step#file:} -m gpu > $log 2>&1 ;;
        smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ;;
        bench) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $log 2>&1 ;;
        bench2) timeout -k 10 300 python bench.py --config 2 --steps 160 --warmup 8 > $log 2>&1 ;;
        slab1) timeout -k 10 300 python bench.py --slab --no-cpu-baseline --steps 20 --warmup 5 > $log 2>&1 ;;
        bench5) timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --steps 20 --warmup 5 > $log 2>&1 ;;
        bench5box) timeout -k 10 400 python bench.py --config 5box --no-cpu-baseline --steps 10 --warmup 3 > $log 2>&1 ;;
        emu*)
            spec=${step#emu}; R=${spec%%-*}; tp=local; dl=0; extra=
            IFS=- read -ra parts <<< "$spec"
            for p in "${parts[@]:1}"; do
                case $p in d*) dl=${p#d} ;; ne) extra=--no-events ;; t*) extra="--timing-every ${p#t}" ;; *) tp=$p ;; esac
            done
            timeout -k 10 300 python bench.py --config 4 --emulate-ranks $R --transport $tp --xfer-delay-us $dl \
                --no-cpu-baseline --steps 100 --warmup 20 $extra > $log 2>&1 ;;
        mp2bench) timeout -k 10 400 python bench.py --gpus 2 --same-device --config 4 --steps 20 --warmup 5 \
                --rank-timeout 360 > $log 2>&1 ;;
        mp4bench|mp8bench) R=${step:2:1}; timeout -k 10 500 python bench.py --gpus $R --same-device --config 4 --steps 10 \
                --warmup 3 --rank-timeout 460 > $log 2>&1 ;;
        rocprof) export TMPDIR=/tmp; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
                -d $OUT/rocprof -o bench -- python3 bench.py --steps 20 --warmup 5 > $log 2>&1 ;;
        py:*) timeout -k 10 300 python tools/${step#py:} > $log 2>&1 ;;
        trace8*) dl=${step#trace8}; dl=${dl#d}; dl=${dl:-0}; export TMPDIR=/tmp
            timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run \
                -- python3 bench.py --config 4 --emulate-ranks 8 --transport ipc --xfer-delay-us $dl --no-cpu-baseline \
                --steps 40 --warmup 10 > $log 2>&1 \
                && python3 tools/timeline_stats.py $OUT/$name/run_kernel_trace.csv 20 > $OUT/${name}_timeline.txt 2>&1 ;;
        tcc) timeout -k 10 600 bash tools/tcc_traffic.sh ${TAG}_$name > $log 2>&1 ;;
        sq) timeout -k 10 500 bash tools/sq_counters.sh $TAG > $log 2>&1 ;;
        shcnt) timeout -k 10 700 bash tools/shift_counters.sh $TAG > $log 2>&1 ;;
        slabtcc) timeout -k 10 900 bash tools/slab_traffic.sh $TAG > $log 2>&1 ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
    rc=$?
    for e in "${envs[@]}"; do unset "${e%%=*}"; done
    if [ $rc -ne 0 ]; then echo "step $spec failed rc $rc"; tail -40 $log; exit $rc; fi
    case $step in
        tests*|mp|smoke|file:*) tail -1 $log ;;
        py:*) tail -25 $log ;;
        trace8*) head -40 $OUT/${name}_timeline.txt ;;
        tcc|sq|shcnt|slabtcc) tail -12 $log ;;
        rocprof) python3 tools/rocprof_timed_mean.py $OUT/rocprof 2>&1 | tail -8 ;;
        *) grep '^{' $log > $OUT/$name.json; summ $OUT/$name.json ;;
    esac
done
