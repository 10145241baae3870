# same-box A/B of the pixel-row weight-gradient forms (MZBA_WGRAD_FORM, mzba_conv_wgrad_set_form): wgrad GPU
# tests, alternating learner minibatches (tools/ab_lib_learner.py), per-launch segment timings
set -e
D=gpurun_out/wgrad_wf2; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > $D/pytest_wgrad.log 2>&1
for f in 2 3 2 3; do MZBA_WGRAD_FORM=$f timeout -k 10 200 python tools/ab_lib_learner.py bf16 >> $D/ab.jsonl; done
timeout -k 10 200 python tools/bench_wgrad_segs.py > $D/segs.jsonl
