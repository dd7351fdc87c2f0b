"""Logging in the reference's formats: the scripts log with
``logging.getLogger(__name__)`` at DEBUG to stdout; these helpers produce the same lines
("Train Epoch: {e} [{n}/{N} ({p:.0f}%)] Loss: {l:.6f}", "Test set: Average loss: ...",
"Initialized the distributed environment: ...") for framework-driven training loops."""
import logging
import sys


def get_logger(name="mi355x_dp", level=logging.DEBUG):
    log = logging.getLogger(name)
    if not log.handlers:
        h = logging.StreamHandler(sys.stdout)
        log.addHandler(h)
    log.setLevel(level)
    return log


def fmt_train(epoch, seen, total, batch_idx, n_batches, loss):
    return "Train Epoch: {} [{}/{} ({:.0f}%)] Loss: {:.6f}".format(epoch, seen, total, 100.0 * batch_idx / n_batches,
                                                                  loss)


def fmt_test(avg_loss, acc):
    return "Test set: Average loss: {:.4f}, Accuracy: {:.2f}\n".format(avg_loss, acc)


def fmt_init(backend, world):
    return "Initialized the distributed environment: '{}' backend on {} nodes. ".format(backend, world)
