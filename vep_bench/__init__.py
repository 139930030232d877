"""Benchmark and check harnesses (not part of the product package): out-of-process gRPC latency
clients, the latency / serving measurements bench.py and tools/bench_serving.py run, the config-5
side loads (RTMP sink, annotation load) and the GPU check of the isolated hub."""
