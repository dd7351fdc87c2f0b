#!/usr/bin/env python
"""Write notebooks/*.ipynb: the workshop's two driver notebooks re-done for
mi355x_dp local mode -- same SageMaker SDK calls (Session, upload_data, PyTorch(...).fit(),
model_data, PyTorchModel(...).deploy(), predictor.predict()), synthetic CIFAR-10 (no network),
the example scripts in examples/.  Cells are plain source so tests/test_notebooks_cpu.py can run
them in order without jupyter.

    python tools/make_notebooks.py
"""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SETUP = '''import os, sys
REPO = os.path.abspath(os.environ.get("MI355X_DP_REPO", ".."))
sys.path.insert(0, REPO)
sys.path.append(os.path.join(REPO, "compat"))   # sagemaker / torchvision / smdistributed stand-ins (last on the path)
EPOCHS = int(os.environ.get("NB_EPOCHS", "{epochs}"))
N_TRAIN = int(os.environ.get("NB_N_TRAIN", "50000"))
N_TEST = int(os.environ.get("NB_N_TEST", "10000"))'''

SESSION = '''import sagemaker
sess = sagemaker.Session()
role = sagemaker.get_execution_role()
bucket = sess.default_bucket()
print(bucket, role)'''

DATA = '''from mi355x_dp.data.cifar import write_synthetic_cifar10
# no network: a synthetic dataset in the official cifar-10-batches-py pickle layout
write_synthetic_cifar10("cifar10-dataset", n_train=N_TRAIN, n_test=N_TEST)
inputs = sess.upload_data(path="cifar10-dataset", key_prefix="datasets/cifar10-dataset")
print(inputs)'''

PREDICT = '''import numpy as np
import torch
import torchvision
import torchvision.transforms as transforms
transform = transforms.Compose([transforms.ToTensor(), transforms.Normalize((0.5, 0.5, 0.5), (0.5, 0.5, 0.5))])
testset = torchvision.datasets.CIFAR10(root="cifar10-dataset", train=False, download=False, transform=transform)
testloader = torch.utils.data.DataLoader(testset, batch_size=4, shuffle=True, num_workers=0)
classes = ("plane", "car", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck")
images, labels = next(iter(testloader))
outputs = predictor.predict(images.numpy())
_, predicted = torch.max(torch.from_numpy(np.array(outputs)), 1)
print("GroundTruth:", " ".join(f"{classes[labels[j]]:>5}" for j in range(4)))
print("Predicted:  ", " ".join(f"{classes[predicted[j]]:>5}" for j in range(4)))
print("PREDICT_SHAPE", tuple(np.asarray(outputs).shape))'''


def md(s):
    return {"cell_type": "markdown", "metadata": {}, "source": s.splitlines(True)}


def code(s):
    return {"cell_type": "code", "execution_count": None, "metadata": {}, "outputs": [], "source": s.splitlines(True)}


def nb(cells):
    return {"cells": cells, "metadata": {"kernelspec": {"display_name": "Python 3", "language": "python",
                                                        "name": "python3"},
                                         "language_info": {"name": "python"}},
            "nbformat": 4, "nbformat_minor": 5}


NB1 = nb([
    md("# Distributed data-parallel training on CPUs (gloo) — mi355x_dp local mode\n\n"
       "The workshop's notebook 1: upload CIFAR-10, train a LeNet with PyTorch DDP on **2 instances** over the "
       "gloo backend, deploy the model and classify four test images. Every SageMaker SDK call is served "
       "locally by `mi355x_dp.sagemaker_local` (job runner with the `SM_*` contract, native launcher, "
       "`model.tar.gz` artifact, in-process endpoint)."),
    code(SETUP.format(epochs=20)),
    code(SESSION),
    md("## Data\nThe container has no network, so a synthetic dataset with CIFAR-10's exact on-disk layout "
       "stands in for the download."),
    code(DATA),
    md("## Train: 2 × `ml.c5.2xlarge`, gloo DDP\n`instance_count=2` becomes two ranks (hosts `algo-1`, `algo-2`); "
       "hyperparameters reach the script as `--key value` arguments."),
    code('''from sagemaker.pytorch import PyTorch
hyperparameters = {"epochs": EPOCHS, "lr": 0.01, "momentum": 0.9, "batch-size": 64, "model-type": "custom",
                   "backend": "gloo"}
estimator = PyTorch(entry_point="train_cifar10_cpu.py", source_dir=os.path.join(REPO, "examples"),
                    output_path=f"s3://{bucket}/jobs/", code_location=f"s3://{bucket}/code/", role=role,
                    instance_count=2, instance_type="ml.c5.2xlarge", framework_version="1.8.0", py_version="py3",
                    hyperparameters=hyperparameters)
estimator.fit({"train": inputs}, wait=True)'''),
    code('print("MODEL_DATA", estimator.model_data)'),
    md("## Deploy and predict"),
    code('''from sagemaker.pytorch import PyTorchModel
model = PyTorchModel(model_data=estimator.model_data, source_dir=os.path.join(REPO, "examples"),
                     entry_point="inference_cpu.py", role=role, framework_version="1.6.0", py_version="py3")
predictor = model.deploy(initial_instance_count=1, instance_type="ml.c5.xlarge")'''),
    code(PREDICT),
    code("predictor.delete_endpoint()"),
])

NB2 = nb([
    md("# Distributed data-parallel training on MI355X with the `smddp` backend\n\n"
       "The workshop's notebook 2 (bonus GPU lab): ResNet-18 on CIFAR-10, global batch 256, 15 epochs, "
       "`distribution={\"smdistributed\": {\"dataparallel\": {\"enabled\": True}}}` on one 8-GPU instance. "
       "Here the job runs one rank per local MI355X; `smddp` is mi355x_dp's native c10d backend (RCCL over "
       "xGMI, optional one/two-shot IPC all-reduce)."),
    code(SETUP.format(epochs=15)),
    code(SESSION),
    code(DATA),
    md("## Train: `ml.p4d.24xlarge`-shaped job → every local MI355X, `smddp`"),
    code('''from sagemaker.pytorch import PyTorch
hyperparameters = {"epochs": EPOCHS, "lr": 0.01, "momentum": 0.9, "batch-size": 256, "backend": "smddp"}
distribution = {"smdistributed": {"dataparallel": {"enabled": True}}}
estimator = PyTorch(entry_point="train_cifar10_smddp.py", source_dir=os.path.join(REPO, "examples"),
                    output_path=f"s3://{bucket}/jobs/", code_location=f"s3://{bucket}/code/", role=role,
                    instance_count=1, instance_type="ml.p4d.24xlarge", framework_version="1.11.0", py_version="py38",
                    distribution=distribution, hyperparameters=hyperparameters)
estimator.fit({"train": inputs}, job_name="pytorch-smddp-dist-cifar10", wait=True)'''),
    code('print("MODEL_DATA", estimator.model_data)'),
    md("## Deploy and predict\nThe checkpoint has DDP's `module.` key prefix; `examples/inference.py` strips it."),
    code('''from sagemaker.pytorch import PyTorchModel
model = PyTorchModel(model_data=estimator.model_data, source_dir=os.path.join(REPO, "examples"),
                     entry_point="inference.py", role=role, framework_version="1.6.0", py_version="py3")
predictor = model.deploy(initial_instance_count=1, instance_type="ml.c5.xlarge")'''),
    code(PREDICT),
    code("predictor.delete_endpoint()"),
])


def main():
    out = os.path.join(ROOT, "notebooks")
    os.makedirs(out, exist_ok=True)
    for name, book in (("1_pytorch_dist_native_cpu.ipynb", NB1), ("2_pytorch_dist_smddp_mi355x.ipynb", NB2)):
        with open(os.path.join(out, name), "w") as f:
            json.dump(book, f, indent=1)
            f.write("\n")
        print("wrote", os.path.join("notebooks", name))


if __name__ == "__main__":
    main()
