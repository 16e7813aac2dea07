# Same targets and variables as the reference Makefile (/root/reference/Makefile:1-191):
#   make pre_process compute_ciderdf compute_evalscores train test
# plus MI355X targets: build (gfx950 extension), test-cpu / test-gpu, bench, and
# NGPU > 1 for data-parallel training (one process per GPU over RCCL).
#
# Label files are .npz (same dataset names as the reference .h5; h5py is not in
# this image); set LABEL_EXT=h5 on a machine with h5py for byte-compatible files.

### Directory Setting
IN_DIR?=input
OUT_DIR?=output
META_DIR=$(OUT_DIR)/metadata
FEAT_DIR=$(OUT_DIR)/feature
MODEL_DIR=$(OUT_DIR)/model

MSRVTT2016_DIR=$(IN_DIR)/msrvtt
MSRVTT2017_DIR=$(IN_DIR)/msrvtt2017
YT2T_DIR=$(IN_DIR)/yt2t

SPLITS=train val test
DATASETS?=msrvtt
LABEL_EXT?=npz
FEAT_EXT?=npz
PY?=python

WORD_COUNT_THRESHOLD?=3
MAX_SEQ_LEN?=30

NGPU?=1
MASTER_PORT?=29511

DATASET?=msrvtt
TRAIN_DATASET?=$(DATASET)
VAL_DATASET?=$(DATASET)
TEST_DATASET?=$(DATASET)
TRAIN_SPLIT?=train
VAL_SPLIT?=val
TEST_SPLIT?=test

LEARNING_RATE?=0.0001
LR_UPDATE?=200
BATCH_SIZE?=64
TRAIN_SEQ_PER_IMG?=20
TEST_SEQ_PER_IMG?=20
RNN_SIZE?=512

PRINT_INTERVAL?=20
MAX_PATIENCE?=50
SAVE_CHECKPOINT_FROM?=1

MAX_EPOCHS?=200
NUM_CHUNKS?=1
BEAM_SIZE?=5

TODAY=20170831
EXP_NAME?=exp_$(DATASET)_$(TODAY)
VAL_LANG_EVAL?=1
TEST_LANG_EVAL?=1
EVAL_METRIC?=CIDEr
START_FROM?=No
MODEL_TYPE?=concat
LOGLEVEL?=INFO

SS_MAX_PROB?=0.25
USE_CST?=0
SCB_CAPTIONS?=20
SCB_BASELINE?=1
USE_RL?=0
USE_RL_AFTER?=0
USE_EOS?=0
USE_MIXER?=0
MIXER_FROM?=-1
SS_K?=100

FEAT1?=resnet
FEAT2?=c3d
FEAT3?=mfcc
FEAT4?=category
FEATS?=$(FEAT1) $(FEAT2) $(FEAT3) $(FEAT4)

TRAIN_ID=$(TRAIN_DATASET)_$(MODEL_TYPE)_$(EVAL_METRIC)_$(BATCH_SIZE)_$(LEARNING_RATE)

ifeq ($(NGPU),1)
LAUNCH=$(PY)
else
LAUNCH=$(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $(NGPU) \
	--master-addr 127.0.0.1 --master-port $(MASTER_PORT)
endif
PREPRO=$(PY) -m cst_captioning_amd.prepro

.PHONY: build test-cpu test-gpu bench bench-scale pre_process standalize_datainfo \
	preprocess_datainfo build_vocab create_sequencelabel convert_datainfo2cocofmt \
	compute_ciderdf compute_evalscores train test

### MI355X-specific
build:
	PYTORCH_ROCM_ARCH=gfx950 $(PY) setup.py build_ext --inplace
test-cpu:
	$(PY) -m pytest tests -x -q -m "not gpu"
test-gpu:
	$(PY) -m pytest tests -x -q -m gpu
bench:
	$(LAUNCH) bench.py --gpus $(NGPU)

###################################################################################################################
pre_process: standalize_datainfo preprocess_datainfo build_vocab create_sequencelabel convert_datainfo2cocofmt

standalize_datainfo: $(foreach d,$(DATASETS),$(patsubst %,$(META_DIR)/$(d)_%_datainfo.json,$(SPLITS)))
$(META_DIR)/msrvtt_%_datainfo.json: $(MSRVTT2016_DIR)/%_videodatainfo.json
	$(PREPRO).standalize $^ $@ --dataset msrvtt2016 --split $*
$(META_DIR)/msrvtt2017_%_datainfo.json: $(MSRVTT2017_DIR)/msrvtt2017_%_videodatainfo.json
	$(PREPRO).standalize $^ $@ --dataset msrvtt2017 --split $* \
		--val2016_json $(MSRVTT2016_DIR)/val_videodatainfo.json
$(META_DIR)/yt2t_%_datainfo.json: $(YT2T_DIR)/naacl15/sents_%_lc_nopunc.txt
	$(PREPRO).standalize $^ $@ --dataset yt2t
$(META_DIR)/tvvtt_%_datainfo.json: $(META_DIR)/v2t2017_infos.json
	$(PREPRO).standalize $^ $@ --dataset tvvtt --split $*

preprocess_datainfo: $(foreach s,$(SPLITS),$(patsubst %,$(META_DIR)/%_$(s)_proprocessedtokens.json,$(DATASETS)))
%_proprocessedtokens.json: %_datainfo.json
	$(PREPRO).tokenize $^ $@

build_vocab: $(patsubst %,$(META_DIR)/%_train_vocab.json,$(DATASETS))
%_train_vocab.json: %_train_proprocessedtokens.json
	$(PREPRO).vocab $< $@ --word_count_threshold $(WORD_COUNT_THRESHOLD)

create_sequencelabel: $(foreach s,$(SPLITS),$(patsubst %,$(META_DIR)/%_$(s)_sequencelabel.$(LABEL_EXT),$(DATASETS)))
.SECONDEXPANSION:
%_sequencelabel.$(LABEL_EXT): $$(firstword $$(subst _, ,$$@))_train_vocab.json %_proprocessedtokens.json
	$(PREPRO).labels $^ $@ --max_length $(MAX_SEQ_LEN)

convert_datainfo2cocofmt: $(foreach s,$(SPLITS),$(patsubst %,$(META_DIR)/%_$(s)_cocofmt.json,$(DATASETS)))
%_cocofmt.json: %_datainfo.json
	$(PREPRO).cocofmt $< $@

compute_ciderdf: $(foreach s,$(SPLITS),$(patsubst %,$(META_DIR)/%_$(s)_ciderdf.pkl,$(DATASETS)))
%_ciderdf.pkl: %_proprocessedtokens.json
	$(PREPRO).ciderdf $^ $@ --output_words --vocab_json $(firstword $(subst _, ,$@))_train_vocab.json

compute_evalscores: $(patsubst %,$(META_DIR)/$(TRAIN_DATASET)_%_evalscores.pkl,$(SPLITS))
%_evalscores.pkl: %_cocofmt.json
	$(PREPRO).evalscores $^ $@ --seq_per_img $(TRAIN_SEQ_PER_IMG) --remove_in_ref

#####################################################################################################################
noop=
space=$(noop) $(noop)

TRAIN_OPT=--beam_size $(BEAM_SIZE) --max_patience $(MAX_PATIENCE) --eval_metric $(EVAL_METRIC) \
	--print_log_interval $(PRINT_INTERVAL) --language_eval $(VAL_LANG_EVAL) --max_epochs $(MAX_EPOCHS) \
	--rnn_size $(RNN_SIZE) --train_seq_per_img $(TRAIN_SEQ_PER_IMG) --test_seq_per_img $(TEST_SEQ_PER_IMG) \
	--batch_size $(BATCH_SIZE) --test_batch_size $(BATCH_SIZE) --learning_rate $(LEARNING_RATE) \
	--lr_update $(LR_UPDATE) --save_checkpoint_from $(SAVE_CHECKPOINT_FROM) --num_chunks $(NUM_CHUNKS) \
	--train_cached_tokens $(META_DIR)/$(TRAIN_DATASET)_train_ciderdf.pkl \
	--ss_k $(SS_K) --use_rl_after $(USE_RL_AFTER) --ss_max_prob $(SS_MAX_PROB) \
	--use_rl $(USE_RL) --use_mixer $(USE_MIXER) --mixer_from $(MIXER_FROM) \
	--use_cst $(USE_CST) --scb_captions $(SCB_CAPTIONS) --scb_baseline $(SCB_BASELINE) \
	--loglevel $(LOGLEVEL) --model_type $(MODEL_TYPE) --use_eos $(USE_EOS) \
	--model_file $@ --start_from $(START_FROM) --result_file $(basename $@)_test.json \
	2>&1 | tee $(basename $@).log

TEST_OPT=--beam_size $(BEAM_SIZE) --language_eval $(VAL_LANG_EVAL) --test_seq_per_img $(TEST_SEQ_PER_IMG) \
	--test_batch_size $(BATCH_SIZE) --loglevel $(LOGLEVEL) --result_file $@

train: $(MODEL_DIR)/$(EXP_NAME)/$(subst $(space),$(noop),$(FEATS))_$(TRAIN_ID).pth
$(MODEL_DIR)/$(EXP_NAME)/$(subst $(space),$(noop),$(FEATS))_$(TRAIN_ID).pth: \
	$(META_DIR)/$(TRAIN_DATASET)_$(TRAIN_SPLIT)_sequencelabel.$(LABEL_EXT) \
	$(META_DIR)/$(VAL_DATASET)_$(VAL_SPLIT)_sequencelabel.$(LABEL_EXT) \
	$(META_DIR)/$(TEST_DATASET)_$(TEST_SPLIT)_sequencelabel.$(LABEL_EXT) \
	$(META_DIR)/$(TRAIN_DATASET)_$(TRAIN_SPLIT)_cocofmt.json \
	$(META_DIR)/$(VAL_DATASET)_$(VAL_SPLIT)_cocofmt.json \
	$(META_DIR)/$(TEST_DATASET)_$(TEST_SPLIT)_cocofmt.json \
	$(META_DIR)/$(TRAIN_DATASET)_$(TRAIN_SPLIT)_evalscores.pkl \
	$(patsubst %,$(FEAT_DIR)/$(TRAIN_DATASET)_$(TRAIN_SPLIT)_%_mp$(NUM_CHUNKS).$(FEAT_EXT),$(FEATS)) \
	$(patsubst %,$(FEAT_DIR)/$(VAL_DATASET)_$(VAL_SPLIT)_%_mp$(NUM_CHUNKS).$(FEAT_EXT),$(FEATS)) \
	$(patsubst %,$(FEAT_DIR)/$(TEST_DATASET)_$(TEST_SPLIT)_%_mp$(NUM_CHUNKS).$(FEAT_EXT),$(FEATS))
	mkdir -p $(MODEL_DIR)/$(EXP_NAME)
	$(LAUNCH) train.py \
		--train_label_h5 $(word 1,$^) \
		--val_label_h5 $(word 2,$^) \
		--test_label_h5 $(word 3,$^) \
		--train_cocofmt_file $(word 4,$^) \
		--val_cocofmt_file $(word 5,$^) \
		--test_cocofmt_file $(word 6,$^) \
		--train_bcmrscores_pkl $(word 7,$^) \
		--train_feat_h5 $(patsubst %,$(FEAT_DIR)/$(TRAIN_DATASET)_$(TRAIN_SPLIT)_%_mp$(NUM_CHUNKS).$(FEAT_EXT),$(FEATS)) \
		--val_feat_h5 $(patsubst %,$(FEAT_DIR)/$(VAL_DATASET)_$(VAL_SPLIT)_%_mp$(NUM_CHUNKS).$(FEAT_EXT),$(FEATS)) \
		--test_feat_h5 $(patsubst %,$(FEAT_DIR)/$(TEST_DATASET)_$(TEST_SPLIT)_%_mp$(NUM_CHUNKS).$(FEAT_EXT),$(FEATS)) \
		$(TRAIN_OPT)

test: $(MODEL_DIR)/$(EXP_NAME)/$(subst $(space),$(noop),$(FEATS))_$(TRAIN_ID)_test.json
$(MODEL_DIR)/$(EXP_NAME)/$(subst $(space),$(noop),$(FEATS))_$(TRAIN_ID)_test.json: \
	$(MODEL_DIR)/$(EXP_NAME)/$(subst $(space),$(noop),$(FEATS))_$(TRAIN_ID).pth \
	$(META_DIR)/$(TEST_DATASET)_$(TEST_SPLIT)_sequencelabel.$(LABEL_EXT) \
	$(META_DIR)/$(TEST_DATASET)_$(TEST_SPLIT)_cocofmt.json \
	$(patsubst %,$(FEAT_DIR)/$(TEST_DATASET)_$(TEST_SPLIT)_%_mp$(NUM_CHUNKS).$(FEAT_EXT),$(FEATS))
	$(LAUNCH) test.py \
		--model_file $(word 1,$^) \
		--test_label_h5 $(word 2,$^) \
		--test_cocofmt_file $(word 3,$^) \
		--test_feat_h5 $(patsubst %,$(FEAT_DIR)/$(TEST_DATASET)_$(TEST_SPLIT)_%_mp$(NUM_CHUNKS).$(FEAT_EXT),$(FEATS)) \
		$(TEST_OPT)

.PRECIOUS: %.pth
.SECONDARY:
