"""The SageMaker training-toolkit environment contract.

Reproduces exactly what the captured job log shows (notebooks/2_pytorch_dist_smddp_gpu.ipynb,
"Training Env" JSON and "Environment variables" block): the ``SM_*`` variables the
reference scripts read in their argparse defaults (cifar10-distributed-smddp-gpu.py:234-237,
KeyError if unset) plus hyperparameters rendered as sorted ``--key value`` CLI args
(``SM_USER_ARGS``).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional


def hyperparameters_to_args(hps: Dict) -> List[str]:
    args = []
    for k in sorted(hps):
        v = hps[k]
        if isinstance(v, bool):
            v = str(v)
        args += [f"--{k}", str(v)]
    return args


def training_env(job_name: str, entry_point: str, hyperparameters: Dict, channels: Dict[str, str], model_dir: str,
                 output_dir: str, input_dir: str, hosts: List[str], current_host: str, num_gpus: int, num_cpus: int,
                 instance_type: str, module_dir: str, distribution: Optional[Dict] = None) -> Dict:
    smddp = bool(distribution and distribution.get("smdistributed", {}).get("dataparallel", {}).get("enabled"))
    addl = {}
    if smddp:
        addl = {"sagemaker_distributed_dataparallel_custom_mpi_options": "",
                "sagemaker_distributed_dataparallel_enabled": True,
                "sagemaker_instance_type": instance_type}
    module_name = os.path.splitext(os.path.basename(entry_point))[0]
    return {
        "additional_framework_parameters": addl,
        "channel_input_dirs": dict(channels),
        "current_host": current_host,
        "framework_module": "mi355x_dp.sagemaker_local.training:main",
        "hosts": list(hosts),
        "hyperparameters": dict(hyperparameters),
        "input_config_dir": os.path.join(input_dir, "config"),
        "input_data_config": {c: {"TrainingInputMode": "File", "S3DistributionType": "FullyReplicated",
                                  "RecordWrapperType": "None"} for c in channels},
        "input_dir": input_dir,
        "is_master": current_host == hosts[0],
        "is_modelparallel_enabled": None,
        "job_name": job_name,
        "log_level": 20,
        "master_hostname": hosts[0],
        "model_dir": model_dir,
        "module_dir": module_dir,
        "module_name": module_name,
        "network_interface_name": "lo",
        "num_cpus": num_cpus,
        "num_gpus": num_gpus,
        "output_data_dir": os.path.join(output_dir, "data"),
        "output_dir": output_dir,
        "output_intermediate_dir": os.path.join(output_dir, "intermediate"),
        "resource_config": {"current_host": current_host, "current_instance_type": instance_type,
                            "current_group_name": "homogeneousCluster", "hosts": list(hosts),
                            "instance_groups": [{"instance_group_name": "homogeneousCluster",
                                                 "instance_type": instance_type, "hosts": list(hosts)}],
                            "network_interface_name": "lo"},
        "user_entry_point": os.path.basename(entry_point),
    }


def env_vars(tenv: Dict) -> Dict[str, str]:
    """Flatten a training env into the SM_* variables (same names/JSON encodings as the toolkit)."""
    j = lambda o: json.dumps(o, separators=(",", ":"), sort_keys=True)  # noqa: E731
    hps = tenv["hyperparameters"]
    e = {
        "SM_HOSTS": j(tenv["hosts"]),
        "SM_NETWORK_INTERFACE_NAME": tenv["network_interface_name"],
        "SM_HPS": j(hps),
        "SM_USER_ENTRY_POINT": tenv["user_entry_point"],
        "SM_FRAMEWORK_PARAMS": j(tenv["additional_framework_parameters"]),
        "SM_RESOURCE_CONFIG": j(tenv["resource_config"]),
        "SM_INPUT_DATA_CONFIG": j(tenv["input_data_config"]),
        "SM_OUTPUT_DATA_DIR": tenv["output_data_dir"],
        "SM_CHANNELS": j(sorted(tenv["channel_input_dirs"])),
        "SM_CURRENT_HOST": tenv["current_host"],
        "SM_MODULE_NAME": tenv["module_name"],
        "SM_LOG_LEVEL": str(tenv["log_level"]),
        "SM_FRAMEWORK_MODULE": tenv["framework_module"],
        "SM_INPUT_DIR": tenv["input_dir"],
        "SM_INPUT_CONFIG_DIR": tenv["input_config_dir"],
        "SM_OUTPUT_DIR": tenv["output_dir"],
        "SM_NUM_CPUS": str(tenv["num_cpus"]),
        "SM_NUM_GPUS": str(tenv["num_gpus"]),
        "SM_MODEL_DIR": tenv["model_dir"],
        "SM_MODULE_DIR": tenv["module_dir"],
        "SM_TRAINING_ENV": j(tenv),
        "SM_USER_ARGS": j(hyperparameters_to_args(hps)),
        "SM_OUTPUT_INTERMEDIATE_DIR": tenv["output_intermediate_dir"],
    }
    for ch, d in tenv["channel_input_dirs"].items():
        e[f"SM_CHANNEL_{ch.upper()}"] = d
    for k, v in hps.items():
        e[f"SM_HP_{k.upper()}"] = v if isinstance(v, str) else j(v)
    return e
