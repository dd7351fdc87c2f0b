"""Minimal local ``boto3`` stand-in: ``boto3.Session().client('sagemaker')`` returns a
client object whose calls are no-ops (the workshop only creates it, nb1)."""


class _Client:
    def __init__(self, service):
        self.service = service

    def __getattr__(self, name):
        def _noop(*a, **k):
            return {}
        return _noop


class Session:
    def __init__(self, *a, **k):
        self.region_name = "local"

    def client(self, service, *a, **k):
        return _Client(service)


def client(service, *a, **k):
    return _Client(service)
