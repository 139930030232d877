"""Prometheus metrics (new: the reference exposed none — SURVEY.md §5 observability row).

Scraped lazily from the native counters: per-camera packets / decoded frames / errors / bytes /
published frames / ingest state, per-worker batches and GPU kernel time, gRPC frame latency.
"""
from __future__ import annotations

import statistics

from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, HistogramMetricFamily


class HubCollector:
    def __init__(self, hub, image_service=None, frontends=None):
        self.hub = hub
        self.svc = image_service
        self.frontends = frontends
        self.consumer = None  # engine.consumer.ConsumerLoop
        self.native = None    # native.RpcServer (main-process native endpoint)

    def collect(self):
        labels = ["camera", "device"]
        pk = CounterMetricFamily("vep_packets", "access units received", labels=labels)
        dec = CounterMetricFamily("vep_decoded_frames", "frames reconstructed + converted", labels=labels)
        errs = CounterMetricFamily("vep_decode_errors", "decode errors", labels=labels)
        byt = CounterMetricFamily("vep_ingest_bytes", "bitstream bytes received", labels=labels)
        run = GaugeMetricFamily("vep_camera_running", "ingest session connected", labels=labels)
        rst = CounterMetricFamily("vep_camera_restarts", "ingest reconnects", labels=labels)
        lat = HistogramMetricFamily("vep_decode_latency_seconds",
                                    "packet arrival -> decoded frame published", labels=labels)
        for name in list(self.hub.cameras):
            try:
                st = self.hub.state(name)
            except KeyError:
                continue
            lv = [name, str(st.get("device"))]
            pk.add_metric(lv, st.get("packets", 0))
            dec.add_metric(lv, st.get("decoded", 0))
            errs.add_metric(lv, st.get("errors", 0))
            byt.add_metric(lv, st.get("bytes_in", 0))
            run.add_metric(lv, 1.0 if st.get("running") else 0.0)
            rst.add_metric(lv, st.get("restart_count", 0))
            hist, bounds = st.get("latency_hist"), st.get("latency_bounds_ms")
            if hist and bounds:
                acc, buckets = 0, []
                for b, c in zip(list(bounds) + [float("inf")], hist):
                    acc += c
                    buckets.append((str(b / 1000.0) if b != float("inf") else "+Inf", acc))
                lat.add_metric(lv, buckets, st.get("latency_sum_ms", 0) / 1000.0)
        yield from (pk, dec, errs, byt, run, rst, lat)
        wb = CounterMetricFamily("vep_worker_batches", "batched decode launches", labels=["device"])
        wf = CounterMetricFamily("vep_worker_frames", "frames decoded by the worker", labels=["device"])
        wg = CounterMetricFamily("vep_worker_gpu_ms", "GPU time of decode batches (ms)", labels=["device"])
        for d, w in zip(self.hub.devices, self.hub.workers):
            wb.add_metric([str(d)], w.batches)
            wf.add_metric([str(d)], w.frames)
            wg.add_metric([str(d)], w.gpu_ms_total)
        yield from (wb, wf, wg)
        try:
            from .._native import native

            ps = native.pinned_pool_stats()
            pool = GaugeMetricFamily("vep_pinned_pool_bytes", "pinned ingest pool reserved bytes")
            pool.add_metric([], ps["bytes_reserved"])
            yield pool
        except Exception:  # noqa: BLE001 — metrics must never fail a scrape
            pass
        if self.consumer is not None:
            st = self.consumer.stats()
            cg = CounterMetricFamily("vep_consumer_gathers", "node consumer batches gathered")
            cg.add_metric([], st["gathers"])
            ce = CounterMetricFamily("vep_consumer_errors", "node consumer batches that failed")
            ce.add_metric([], st["errors"])
            yield from (cg, ce)
            if st["gather_ms_p50"] is not None:
                g = GaugeMetricFamily("vep_consumer_gather_ms", "steady-state gather time per batch",
                                      labels=["quantile"])
                g.add_metric(["0.5"], st["gather_ms_p50"])
                g.add_metric(["0.99"], st["gather_ms_p99"])
                yield g
        if self.svc is not None:
            served = CounterMetricFamily("vep_grpc_frames_served", "VideoLatestImage frames sent",
                                         labels=["process"])
            served.add_metric(["main"], self.svc.frames_served)
            if self.frontends is not None:
                served.add_metric(["serving"], self.frontends.frames_served())
            nst = self.native.stats() if self.native is not None else None
            if nst is not None:
                served.add_metric(["native"], nst["frames_served"])
            yield served
            if nst is not None:
                g = GaugeMetricFamily("vep_native_frame_latency_ms", "native endpoint: request -> response queued",
                                      labels=["quantile"])
                g.add_metric(["0.5"], nst["p50_ms"])
                g.add_metric(["0.99"], nst["p99_ms"])
                yield g
                c = GaugeMetricFamily("vep_native_connections", "native endpoint open connections")
                c.add_metric([], nst["connections_open"])
                yield c
            lat = list(self.svc.latencies_ms)
            if lat:
                g = GaugeMetricFamily("vep_grpc_frame_latency_ms", "server-side frame latency",
                                      labels=["quantile"])
                s = sorted(lat)
                g.add_metric(["0.5"], statistics.median(s))
                g.add_metric(["0.99"], s[max(0, int(len(s) * 0.99) - 1)])
                yield g


class Metrics:
    def __init__(self, hub, image_service=None, frontends=None):
        self.registry = CollectorRegistry()
        self.collector = HubCollector(hub, image_service, frontends)
        self.registry.register(self.collector)

    @property
    def native(self):
        return self.collector.native

    @native.setter
    def native(self, srv):
        self.collector.native = srv

    @property
    def consumer(self):
        return self.collector.consumer

    @consumer.setter
    def consumer(self, loop):
        self.collector.consumer = loop

    def render(self):
        return generate_latest(self.registry), CONTENT_TYPE_LATEST
