"""MNTD (Meta Neural Trojan Detection) "cloud-security" workflow bundled with the reference
(notebooks/code/{utils_*,meta_classifier,run_meta_cpu,train_basic_*}.py, model_lib/):
target-model family, trojan generation, shadow-model generation (serial and task-parallel),
meta-classifier (+ one-class) training with device-resident checkpoint banks."""
from .data import BackdoorDataset, load_dataset_setting  # noqa: F401
from .meta import (CheckpointBank, MetaClassifier, MetaClassifierOC, epoch_meta_eval, epoch_meta_eval_oc,  # noqa
                   epoch_meta_train, epoch_meta_train_oc, load_model_setting)
from .models import AudioRNN, CIFARCNN, MNISTCNN, RTNLPCNN, mel_filterbank  # noqa: F401
from .train import eval_model, generate, train_model  # noqa: F401
