#!/bin/bash
# End-to-end training on synthetic MSR-VTT-shaped data through the reference
# CLI (train.py): XE warm-up, then SCST (greedy baseline) and CST (SCB*, sample
# baseline) fine-tuning from the XE checkpoint; beam-5 validation each epoch.
# Usage: bash scripts/e2e_train.sh OUT_DIR [extra flags]
# Checkpoints go to $E2E_CKPT (default /tmp/e2e_ckpt); logs, histories and
# test results are copied to OUT_DIR.
set -o pipefail
DEST=${1:-gpurun_out/e2e}; shift
OUT=${E2E_CKPT:-/tmp/e2e_ckpt}
mkdir -p $OUT $DEST
trap 'cp $OUT/*.json $OUT/*.log $DEST/ 2>/dev/null' EXIT
COMMON="--synthetic msrvtt --synthetic_videos ${E2E_VIDEOS:-2000} --synthetic_vocab ${E2E_VOCAB:-4000} \
  --batch_size 64 --train_seq_per_img 20 --test_seq_per_img 20 --test_batch_size 64 --beam_size 5 \
  --language_eval 1 --eval_metric CIDEr --save_checkpoint_from 1 --print_log_interval 20 \
  --loglevel INFO --max_patience 50 $@"
python train.py $COMMON --max_epochs ${E2E_XE_EPOCHS:-8} --learning_rate 2e-3 \
  --model_file $OUT/xe.pth --result_file $OUT/xe_test.json > $OUT/xe.log 2>&1 || exit $?
python train.py $COMMON --max_epochs ${E2E_RL_EPOCHS:-12} --learning_rate 2e-4 \
  --use_rl 1 --use_cst 0 --use_mixer 1 --mixer_from 1 --use_eos 1 --start_from $OUT/xe.pth \
  --model_file $OUT/scst.pth --result_file $OUT/scst_test.json > $OUT/scst.log 2>&1 || exit $?
python train.py $COMMON --max_epochs ${E2E_RL_EPOCHS:-12} --learning_rate 2e-4 \
  --use_rl 1 --use_cst 1 --use_mixer 1 --mixer_from 1 --scb_baseline 2 --scb_captions 20 \
  --use_eos 1 --start_from $OUT/xe.pth \
  --model_file $OUT/cst.pth --result_file $OUT/cst_test.json > $OUT/cst.log 2>&1 || exit $?
