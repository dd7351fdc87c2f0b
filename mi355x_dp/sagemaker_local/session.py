"""Local stand-in for ``sagemaker.Session`` + S3 (reference nb1:35-75).

``s3://bucket/key`` URIs map onto a directory tree under ``MI355X_DP_S3_ROOT``
(default ``~/.mi355x_dp/s3``): ``upload_data`` copies there and returns the URI the
estimator later resolves back to a local path for its ``train`` channel.
"""
from __future__ import annotations

import os
import shutil

DEFAULT_ROLE = "arn:aws:iam::000000000000:role/mi355x-dp-local"


def s3_root() -> str:
    return os.path.abspath(os.path.expanduser(os.environ.get("MI355X_DP_S3_ROOT", "~/.mi355x_dp/s3")))


def s3_to_local(uri: str) -> str:
    if not uri.startswith("s3://"):
        return os.path.abspath(uri)
    return os.path.join(s3_root(), uri[len("s3://"):])


def local_to_s3(path: str) -> str:
    path = os.path.abspath(path)
    root = s3_root()
    if path.startswith(root + os.sep):
        return "s3://" + path[len(root) + 1:]
    return path


class Session:
    def __init__(self, boto_session=None, **kwargs):
        self.boto_session = boto_session
        self._bucket = os.environ.get("MI355X_DP_DEFAULT_BUCKET", "sagemaker-local-mi355x")

    def default_bucket(self) -> str:
        os.makedirs(os.path.join(s3_root(), self._bucket), exist_ok=True)
        return self._bucket

    def upload_data(self, path: str, bucket: str = None, key_prefix: str = "data", **kwargs) -> str:
        bucket = bucket or self.default_bucket()
        dst = os.path.join(s3_root(), bucket, key_prefix)
        if os.path.isdir(path):
            shutil.copytree(path, dst, dirs_exist_ok=True)
        else:
            os.makedirs(dst, exist_ok=True)
            shutil.copy2(path, dst)
        return f"s3://{bucket}/{key_prefix}"

    def download_data(self, path: str, bucket: str, key_prefix: str = "", **kwargs):
        src = os.path.join(s3_root(), bucket, key_prefix)
        shutil.copytree(src, path, dirs_exist_ok=True)
        return path

    @property
    def boto_region_name(self):
        return "local"


def get_execution_role(sagemaker_session=None) -> str:
    return DEFAULT_ROLE
