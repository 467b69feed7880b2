#!/bin/bash
# One parametrised GPU-box session (replaces the per-session one-off scripts of rounds 1-3).
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Steps (each under its own time limit; output in gpurun_out/<tag>/<step>.log; the first
# crash / timeout / abort ends the session, a plain test failure (rc 1) does not):
#   smoke            __graft_entry__.smoke()
#   tests            the whole GPU suite (pytest -m gpu, incl. slow)
#   tests_fast       pytest -m "gpu and not slow"
#   tests:<expr>     pytest -m gpu -k <expr>
#   probe:<lib>:<expr>  the same against another build of the GPU library (fpnn_amd/<lib>, loaded
#                    through FPNN_AES_GPU_LIB), e.g. a tools/probe/*.patch build
#   guard            tests/cpp/guard_pages.cpp: ragged encrypts over arrays abutting unmapped pages
#   guard_audit      the same through the address-audit build (libfpnn_aes_gpu_audit.so)
#   audit:<expr>     pytest -m gpu -k <expr> through the address-audit build
#   bench            python bench.py (the contract line)
#   bench_driver     bench.py three times with the driver's arguments (--steps 20 --warmup 5)
#   bench_trace      bench.py under rocprofv3 --kernel-trace --stats (profiles the line's kernels)
#   bench_pmc        bench.py under the five PMC passes (HBM bytes, LDS, VALU, waits, EA read sizes)
#   configs          tools/bench_configs.py --no-host, every device config (steady-state medians)
#   configs:<list>   the same for a comma list, e.g. configs:C4,R1
#   host             tools/bench_configs.py --configs C2,S1 with the host / PCIe legs
#   s1               S1 (stream host frames) twice with the host-stats breakdown
#   ab:<VAR>:<list>[:<vals>]  same-box A/B of a dispatch knob: the configs with VAR=0, VAR=1 (or each of
#                    the comma list vals), twice
#   k0s              tools/bench_k0s.py (resident small-call servers beside batch kernels, both ways)
#   iomulti          tools/bench_io_multi.py (echoes/s through FPNN's IO plumbing: reference vs batched)
#   ldsprobe         tools/probe/lds_ceiling (compute-only LDS ceilings: b32 vs b64 images, bare loops)
#   timer            tools/timer_probe.py (bench.py vs bench_configs timing loops, one process)
#   abframes[:<lib>] tools/ab_frames.py (short-frame encrypt: K2s vs K2 on Q1 / Q1s / Q1w, alternating),
#                    optionally through another build of the GPU library (fpnn_amd/<lib>)
#   percall          tools/bench_percall.py (C1's shape: per-call drop-in vs the reference)
#   percall_trace    rocprofv3 kernel + HIP API trace of 1000 per-call encrypts + decrypts
#   trace:<cfg>      rocprofv3 kernel trace (no counters) of one bench_configs config
#   prof:<cfg>       rocprofv3 trace + 5 PMC passes of one bench_configs config (or ECDH)
#   ecdh             tools/bench_ecdh.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PASSES="FETCH_SIZE|WRITE_SIZE|SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES|SQ_WAIT_INST_LDS,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE|TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum"

run() {  # run <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -E '^\{|passed|failed|error' "$OUT/$name.log" | tail -3 | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -8 "$OUT/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}

pmc_passes() {  # pmc_passes <dir> <kernel regex> <cmd...>
  local dir=$1 rx=$2; shift 2
  mkdir -p "$OUT/$dir"
  run "$dir/trace" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$dir/trace" -o run -- "$@"
  local i=0 g
  IFS="|" read -ra PG <<< "$PASSES"
  for g in "${PG[@]}"; do
    i=$((i+1))
    run "$dir/pmc$i" 120 rocprofv3 --kernel-trace --pmc ${g//,/ } --kernel-include-regex "$rx" --output-format csv \
      -d "$OUT/$dir/pmc$i" -o run -- "$@"
  done
}

percall_exe() {
  g++ -std=c++11 -O2 -I include oracle/percall.cpp -o "$OUT/percall_gpu" -L fpnn_amd -lfpnn_aes \
    -Wl,-rpath,"$PWD/fpnn_amd" || exit 3
}

for step in "$@"; do
  case "$step" in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1100 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread ;;
    tests_fast) run tests_fast 600 python -u -m pytest tests -q -m "gpu and not slow" -x --timeout 120 --timeout-method thread ;;
    tests:*) run "tests_k" 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -k "${step#tests:}" ;;
    probe:*) spec=${step#probe:}; lib=${spec%%:*}
      FPNN_AES_GPU_LIB=$PWD/fpnn_amd/$lib run "probe_${lib%.so}" 600 python -u -m pytest tests -q -m gpu \
        --timeout 300 --timeout-method thread -k "${spec#*:}" ;;
    guard|guard:*|guard_audit|guard_audit:*)  # (:<args> comma-separated, e.g. guard_audit:--malloc)
      [ -x "$OUT/guard_pages" ] || { gcc -O2 -fPIC -c oracle/aes_oracle.c -o "$OUT/aes_oracle.o" &&
        g++ -std=c++14 -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tests/cpp/guard_pages.cpp "$OUT/aes_oracle.o" \
          -o "$OUT/guard_pages" -L fpnn_amd -lfpnn_aes -Wl,-rpath,"$PWD/fpnn_amd" -L/opt/rocm/lib -lamdhip64 \
          -Wl,-rpath,/opt/rocm/lib -pthread || exit 3; }
      gname=${step%%:*}; gargs=""; [ "$gname" != "$step" ] && gargs=${step#*:}
      glog=$gname${gargs:+_${gargs//[^a-z]/}}
      if [ "$gname" = guard ]; then run "$glog" 300 "$OUT/guard_pages" ${gargs//,/ }
      else FPNN_AES_GPU_LIB=$PWD/fpnn_amd/libfpnn_aes_gpu_audit.so run "$glog" 300 "$OUT/guard_pages" ${gargs//,/ }; fi ;;
    audit:*) FPNN_AES_GPU_LIB=$PWD/fpnn_amd/libfpnn_aes_gpu_audit.so run audit 900 python -u -m pytest tests -q -m gpu \
        --timeout 300 --timeout-method thread -p no:cacheprovider -k "${step#audit:}" ;;
    bench) run bench 300 python -u bench.py ;;
    bench_driver) for i in 1 2 3; do  # the driver's own arguments (BENCH_rNN.json: --steps 20 --warmup 5)
        run "bench_driver_$i" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      done ;;
    bench_trace) mkdir -p "$OUT/bench_trace"  # (bench_pmc's own trace pass goes to bench_prof/trace)
      run bench_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_trace" -o run -- \
        python3 bench.py --no-cpu-baseline ;;
    bench_pmc) pmc_passes bench_prof 'cfb_' python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 ;;
    configs) run configs 700 python -u tools/bench_configs.py --reps 3 --no-host ;;
    configs:*) run "configs_${step#configs:}" 600 python -u tools/bench_configs.py --reps 3 --no-host --configs "${step#configs:}" ;;
    host) run host 600 python -u tools/bench_configs.py --reps 3 --configs C2,S1 ;;
    s1) for i in 1 2; do
        FPNN_AES_HOST_STATS=1 run "s1_$i" 300 python -u tools/bench_configs.py --reps 3 --configs S1
      done ;;
    ab:*) spec=${step#ab:}; var=${spec%%:*}; rest=${spec#*:}; cfgs=${rest%%:*}; vals=0,1
      [ "$rest" != "$cfgs" ] && vals=${rest#*:}
      for i in 1 2; do for v in ${vals//,/ }; do
        env "$var=$v" timeout -k 10 300 python -u tools/bench_configs.py --reps 3 --no-host --configs "$cfgs" \
          > "$OUT/ab_${var}_${v}_$i.log" 2>&1 || { echo "ab $var=$v failed"; tail -5 "$OUT/ab_${var}_${v}_$i.log"; exit 3; }
        echo "   $var=$v #$i: $(grep -h '^{"configs"' "$OUT/ab_${var}_${v}_$i.log" | cut -c1-700)"
      done; done ;;
    timer) run timer 300 python -u tools/timer_probe.py ;;
    abframes) run abframes 600 python -u tools/ab_frames.py ;;
    abframes:*) lib=${step#abframes:}; FPNN_AES_GPU_LIB=$PWD/fpnn_amd/$lib run "abframes_${lib%.so}" 600 python -u tools/ab_frames.py ;;
    ldsprobe) run lds_ceiling 300 tools/probe/lds_ceiling ;;
    iomulti) run iomulti 600 python -u tools/bench_io_multi.py ;;
    k0s) run k0s 600 python -u tools/bench_k0s.py ;;  # (built on the CPU side: hipcc ... lds_ceiling.hip)
    percall) run percall 300 python -u tools/bench_percall.py ;;
    percall_trace) percall_exe
      run percall_trace 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv \
        -d "$OUT/percall_prof" -o run -- "$OUT/percall_gpu" 1000 1024 ;;
    trace:*) c=${step#trace:}; mkdir -p "$OUT/trace_$c"
      run "trace_$c/trace" 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
        -d "$OUT/trace_$c/trace" -o run -- python3 tools/bench_configs.py --configs "$c" --reps 1 ;;
    prof:ECDH) pmc_passes prof_ECDH 'k_ecdh' python3 tools/bench_ecdh.py --curves secp256k1 --no-cpu --reps 3 ;;
    prof:*) c=${step#prof:}; pmc_passes "prof_$c" 'cfb_' python3 tools/bench_configs.py --configs "$c" --no-host --reps 3 ;;
    ecdh) run ecdh 300 python -u tools/bench_ecdh.py ;;
    diag_dropin)  # the drop-in receiver on one framing case with the HIP runtime's log on
      AMD_LOG_LEVEL=3 run diag_framing 120 oracle/_ref/framing_dropin tools/probe/case0.bin "$OUT/case0.jsonl"
      AMD_LOG_LEVEL=3 run diag_echo 120 oracle/_ref/io_echo_dropin 0 32 20 1024 1
      run diag_echo_nolog 120 oracle/_ref/io_echo_dropin 0 32 2000 1024 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done $(date +%T)"
