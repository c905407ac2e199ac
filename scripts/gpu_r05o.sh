# Round-5 (o): is the blit D2H of torch processes the bundled HIP runtime or torch itself, and which
# runtime knob restores SDMA (copy times: SDMA 7.06 ms, blit ~7.4 ms per 402 MB)?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/o
mkdir -p $O
run() { # name env-assignments mode
  env $2 timeout -k 10 120 python3 scripts/d2h_probe_torch.py $3 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; return 1; }
  echo "== $1: $(grep -E '^(C stream 1|E caller)' $O/$1.log | tr '\n' ' ')"
}
run plain "A=0" plain || exit 11
run torchlib "A=0" torchlib || exit 11
run torch "A=0" torch || exit 11
run torch_bet1 "GPU_BLIT_ENGINE_TYPE=1" torch || exit 11
run torch_bet2 "GPU_BLIT_ENGINE_TYPE=2" torch || exit 11
run torch_fbcs0 "GPU_FORCE_BLIT_COPY_SIZE=0" torch || exit 11
run torch_log "AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x7fffffff" torch || true
grep -i -E "hsa copy|blit|sdma|copy engine" $O/torch_log.log | head -40 > $O/torch_log_copies.txt
head -40 $O/torch_log_copies.txt
run plain_log "AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x7fffffff" plain || true
grep -i -E "hsa copy|blit|sdma|copy engine" $O/plain_log.log | head -40 > $O/plain_log_copies.txt
head -20 $O/plain_log_copies.txt
rm -f $O/torch_log.log $O/plain_log.log
exit 0
