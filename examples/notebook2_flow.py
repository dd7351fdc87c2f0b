#!/usr/bin/env python
"""Notebook-2 flow end to end on local MI355X hardware: synthetic CIFAR-10 on "S3", a
smddp-distributed PyTorch estimator fit(), the model artifact, then deploy() + predict() --
the same SageMaker Python SDK calls the workshop notebook makes (compat `sagemaker` package).

    python examples/notebook2_flow.py --epochs 1 --n-train 4096
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.append(os.path.join(ROOT, "compat"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--n-train", type=int, default=4096)
    ap.add_argument("--n-test", type=int, default=1000)
    ap.add_argument("--workdir", default="nb2_work")
    a = ap.parse_args()
    import numpy as np
    import sagemaker
    from sagemaker.pytorch import PyTorch, PyTorchModel
    from mi355x_dp.data.cifar import write_synthetic_cifar10

    os.makedirs(a.workdir, exist_ok=True)
    data = os.path.abspath(os.path.join(a.workdir, "data"))  # channel root holding cifar-10-batches-py/
    write_synthetic_cifar10(data, n_train=a.n_train, n_test=a.n_test)
    sess = sagemaker.Session()
    role = sagemaker.get_execution_role()
    inputs = sess.upload_data(path=data, key_prefix="data/cifar10")
    est = PyTorch(entry_point="train_cifar10_smddp.py", source_dir=os.path.join(ROOT, "examples"), role=role,
                  instance_count=1, instance_type="ml.p4d.24xlarge", framework_version="1.11.0", py_version="py38",
                  hyperparameters={"epochs": a.epochs, "lr": 0.01, "momentum": 0.9, "batch-size": 256,
                                   "backend": "smddp"},
                  distribution={"smdistributed": {"dataparallel": {"enabled": True}}},
                  output_path=os.path.abspath(os.path.join(a.workdir, "out")))
    est.fit({"train": inputs}, job_name="nb2-smddp-job")
    print("MODEL_DATA", est.model_data)
    model = PyTorchModel(model_data=est.model_data, role=role, entry_point="inference.py",
                         source_dir=os.path.join(ROOT, "examples"), framework_version="1.6.0")
    predictor = model.deploy(initial_instance_count=1, instance_type="ml.c5.xlarge")
    out = predictor.predict(np.random.rand(4, 3, 32, 32).astype("float32"))
    print("PREDICT_SHAPE", tuple(np.asarray(out).shape))


if __name__ == "__main__":
    main()
