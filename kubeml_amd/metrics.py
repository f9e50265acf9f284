"""Prometheus metrics — same names/labels as the reference's parameter server
(ml/pkg/ps/metrics.go:18-81): ``kubeml_job_{validation_loss, validation_accuracy,
train_loss, parallelism, epoch_duration_seconds}{jobid}`` and
``kubeml_job_running_total{type}``, exposed on ``:8080/metrics``
(ps/parameter_server.go:57-66).

MI355X additions: per-job throughput ``kubeml_worker_images_per_second``,
collective time ``kubeml_allreduce_seconds`` and device memory ``kubeml_hbm_bytes``.
A private registry keeps tests independent of the process-global default one.
"""
from __future__ import annotations

import threading

from prometheus_client import CollectorRegistry, Gauge, generate_latest
from prometheus_client.exposition import CONTENT_TYPE_LATEST

from .api.types import MetricUpdate


class Metrics:
    def __init__(self):
        self.registry = CollectorRegistry()
        r = self.registry
        self.val_loss = Gauge("kubeml_job_validation_loss", "Validation loss of the job", ["jobid"], registry=r)
        self.val_acc = Gauge("kubeml_job_validation_accuracy", "Validation accuracy of the job", ["jobid"],
                             registry=r)
        self.train_loss = Gauge("kubeml_job_train_loss", "Train loss of the job", ["jobid"], registry=r)
        self.parallelism = Gauge("kubeml_job_parallelism", "Parallelism of the job", ["jobid"], registry=r)
        self.epoch_duration = Gauge("kubeml_job_epoch_duration_seconds", "Duration of the last epoch", ["jobid"],
                                    registry=r)
        self.running = Gauge("kubeml_job_running_total", "Number of running jobs", ["type"], registry=r)
        self.img_s = Gauge("kubeml_worker_images_per_second", "Training throughput of the job (all workers)",
                           ["jobid"], registry=r)
        self.allreduce = Gauge("kubeml_allreduce_seconds", "Time spent in K-AVG/gradient collectives last epoch",
                               ["jobid"], registry=r)
        self.hbm = Gauge("kubeml_hbm_bytes", "Device memory allocated by the job's workers", ["jobid"], registry=r)
        self._lock = threading.Lock()
        self._per_job = (self.val_loss, self.val_acc, self.train_loss, self.parallelism, self.epoch_duration,
                         self.img_s, self.allreduce, self.hbm)

    # reference: updateMetrics (metrics.go:110-133)
    def update(self, job_id: str, m: MetricUpdate):
        with self._lock:
            self.val_loss.labels(job_id).set(m.validations_loss)
            self.val_acc.labels(job_id).set(m.accuracy)
            self.train_loss.labels(job_id).set(m.train_loss)
            self.parallelism.labels(job_id).set(m.parallelism)
            self.epoch_duration.labels(job_id).set(m.epoch_duration)

    def update_extra(self, job_id: str, images_per_second=None, allreduce_seconds=None, hbm_bytes=None):
        with self._lock:
            if images_per_second is not None:
                self.img_s.labels(job_id).set(images_per_second)
            if allreduce_seconds is not None:
                self.allreduce.labels(job_id).set(allreduce_seconds)
            if hbm_bytes is not None:
                self.hbm.labels(job_id).set(hbm_bytes)

    # reference: clearMetrics (metrics.go:90-96)
    def clear(self, job_id: str):
        with self._lock:
            for g in self._per_job:
                try:
                    g.remove(job_id)
                except KeyError:
                    pass

    def task_started(self, kind: str = "train"):
        self.running.labels(kind).inc()

    def task_finished(self, kind: str = "train"):
        self.running.labels(kind).dec()

    def exposition(self) -> bytes:
        return generate_latest(self.registry)

    content_type = CONTENT_TYPE_LATEST


def latest_metrics(history) -> MetricUpdate:
    """MetricUpdate from the tail of a JobHistory (reference getLatestMetrics,
    ml/pkg/train/util.go:188-206: zeros for lists still empty)."""
    last = lambda xs: float(xs[-1]) if xs else 0.0
    return MetricUpdate(validations_loss=last(history.validation_loss), accuracy=last(history.accuracy),
                        train_loss=last(history.train_loss), parallelism=last(history.parallelism),
                        epoch_duration=last(history.epoch_duration))
