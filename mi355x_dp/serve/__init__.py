"""Model serving: the SageMaker PyTorch inference-toolkit contract, locally.

The user's ``inference.py`` supplies ``model_fn(model_dir)`` (reference
notebooks/code/inference.py:28-34) and may override ``input_fn`` /
``predict_fn`` / ``output_fn``; the defaults match the toolkit: a numpy (``.npy``)
or JSON payload becomes a tensor, ``predict_fn`` runs ``model(x)`` under
``torch.no_grad()``, and the result is serialised back (numpy array).  The model
archive is ``model.tar.gz`` from the training job.  ``Predictor.predict`` works
in-process or over HTTP (``http=True`` spins up a local HTTP endpoint).
"""
from __future__ import annotations

import importlib.util
import io
import json
import os
import sys
import tarfile
import tempfile
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np
import torch

NPY = "application/x-npy"
JSON = "application/json"


def default_input_fn(body: bytes, content_type: str = NPY):
    if content_type == NPY:
        return torch.from_numpy(np.load(io.BytesIO(body), allow_pickle=False))
    if content_type == JSON:
        return torch.tensor(json.loads(body))
    raise ValueError(f"unsupported content type {content_type}")


def default_predict_fn(data, model):
    dev = next(model.parameters()).device if any(True for _ in model.parameters()) else torch.device("cpu")
    with torch.no_grad():
        return model(data.to(dev))


def default_output_fn(prediction, accept: str = NPY):
    if isinstance(prediction, torch.Tensor):
        prediction = prediction.detach().float().cpu().numpy()
    if accept == NPY:
        buf = io.BytesIO()
        np.save(buf, np.asarray(prediction), allow_pickle=False)
        return buf.getvalue()
    if accept == JSON:
        return json.dumps(np.asarray(prediction).tolist()).encode()
    raise ValueError(f"unsupported accept type {accept}")


class ModelServer:
    def __init__(self, module, model_dir: str, device: str = "cpu"):
        self.module = module
        self.model_dir = model_dir
        model_fn = getattr(module, "model_fn", None)
        if model_fn is None:
            raise AttributeError("inference entry point must define model_fn(model_dir)")
        self.model = model_fn(model_dir)
        if device != "cpu" and torch.cuda.is_available():
            self.model = self.model.to(device)
        self.model.eval()
        self.input_fn = getattr(module, "input_fn", default_input_fn)
        self.predict_fn = getattr(module, "predict_fn", default_predict_fn)
        self.output_fn = getattr(module, "output_fn", default_output_fn)

    def invoke(self, body: bytes, content_type: str = NPY, accept: str = NPY) -> bytes:
        data = self.input_fn(body, content_type)
        pred = self.predict_fn(data, self.model)
        return self.output_fn(pred, accept)


def _load_module(path: str):
    spec = importlib.util.spec_from_file_location(os.path.splitext(os.path.basename(path))[0], path)
    mod = importlib.util.module_from_spec(spec)
    sys.path.insert(0, os.path.dirname(path))
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.path.pop(0)
    return mod


def extract_model(model_data: str) -> str:
    from mi355x_dp.sagemaker_local.session import s3_to_local
    path = s3_to_local(model_data) if model_data.startswith("s3://") else model_data
    if os.path.isdir(path):
        return path
    out = tempfile.mkdtemp(prefix="mi355x_dp_model_")
    with tarfile.open(path, "r:gz") as tf:
        for m in tf.getmembers():  # refuse path traversal
            if m.name.startswith("/") or ".." in m.name.split("/"):
                raise ValueError(f"unsafe member {m.name} in model archive")
        tf.extractall(out)
    return out


def load_model_server(model_data: str, entry_point: str, source_dir=None, device: str = "cpu") -> ModelServer:
    script = os.path.join(source_dir, entry_point) if source_dir else entry_point
    return ModelServer(_load_module(script), extract_model(model_data), device)


class _Handler(BaseHTTPRequestHandler):
    server_obj: ModelServer = None

    def do_GET(self):  # /ping
        self.send_response(200 if self.path == "/ping" else 404)
        self.end_headers()

    def do_POST(self):  # /invocations
        n = int(self.headers.get("Content-Length", "0"))
        body = self.rfile.read(n)
        try:
            out = self.server_obj.invoke(body, self.headers.get("Content-Type", NPY), self.headers.get("Accept", NPY))
            self.send_response(200)
            self.send_header("Content-Type", self.headers.get("Accept", NPY))
            self.end_headers()
            self.wfile.write(out)
        except Exception as e:  # pragma: no cover - error path
            self.send_response(500)
            self.end_headers()
            self.wfile.write(str(e).encode())

    def log_message(self, *a):
        pass


class Predictor:
    """``predictor.predict(images)`` -> numpy logits (reference nb1:208-209)."""

    def __init__(self, server: ModelServer, endpoint_name: str = "local-endpoint", http: bool = False):
        self.server = server
        self.endpoint_name = endpoint_name
        self._httpd = None
        self.url = None
        if http:
            handler = type("H", (_Handler,), {"server_obj": server})
            self._httpd = ThreadingHTTPServer(("127.0.0.1", 0), handler)
            threading.Thread(target=self._httpd.serve_forever, daemon=True).start()
            self.url = f"http://127.0.0.1:{self._httpd.server_address[1]}"

    def predict(self, data, initial_args=None):
        if isinstance(data, torch.Tensor):
            data = data.detach().cpu().numpy()
        buf = io.BytesIO()
        np.save(buf, np.asarray(data), allow_pickle=False)
        if self._httpd is not None:
            import urllib.request
            req = urllib.request.Request(self.url + "/invocations", data=buf.getvalue(),
                                         headers={"Content-Type": NPY, "Accept": NPY})
            out = urllib.request.urlopen(req).read()
        else:
            out = self.server.invoke(buf.getvalue(), NPY, NPY)
        return np.load(io.BytesIO(out), allow_pickle=False)

    def delete_endpoint(self, *a, **k):
        if self._httpd is not None:
            self._httpd.shutdown()
            self._httpd = None

    def delete_model(self, *a, **k):
        pass
