# wgrad ablation builds (numerically wrong by construction; timing only): libmzba_abl1.so = no next-stage global
# loads, libmzba_abl3.so = no per-tap B fragment reloads; per-launch timings beside the product build
set -e
D=gpurun_out/wgrad_abl; mkdir -p $D
for L in libmzba.so libmzba_abl1.so libmzba_abl3.so libmzba.so; do
  MZBA_LIB=muzero-breakout_amd/mzba/$L timeout -k 10 200 python tools/bench_wgrad_segs.py | sed "s/^{/{\"lib\": \"$L\", /" >> $D/segs.jsonl
done
