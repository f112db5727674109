"""python -m devspace_amd.localkube up --state DIR [--port P] [--gpus N] [--kubeconfig PATH] [--context NAME] [--tls]
                                   [--throttle-first K --retry-after S] [--partition spx|dpx|qpx|cpx]
                                   [--nps nps1|nps2] [--resource-strategy single|mixed] [--unhealthy K]"""
import argparse
import os
import signal
import sys
import threading

from .cluster import LocalCluster


def main(argv=None):
    ap = argparse.ArgumentParser(prog="devspace_amd.localkube")
    sub = ap.add_subparsers(dest="cmd", required=True)
    up = sub.add_parser("up", help="run the local cluster in the foreground")
    up.add_argument("--state", required=True)
    up.add_argument("--port", type=int, default=0)
    up.add_argument("--gpus", type=int, default=None)
    up.add_argument("--kubeconfig", default="")
    up.add_argument("--namespace", default="default")
    up.add_argument("--context", default="devspace-local", help="kube context name (e.g. minikube)")
    up.add_argument("--tls", action="store_true", help="https + wss with client certificates")
    up.add_argument("--throttle-first", type=int, default=0,
                    help="fault switch: answer the first K requests of every (verb, resource) with 429")
    up.add_argument("--retry-after", type=int, default=1, help="Retry-After seconds of the throttled answers")
    up.add_argument("--pull-seconds", type=float, default=0.0,
                    help="slow-pull mode: every image takes this long to pull the first time (Pulling events)")
    up.add_argument("--partition", default="spx", choices=("spx", "dpx", "qpx", "cpx"),
                    help="compute partition mode of the node's GPUs (CPX: 8 devices per MI355X)")
    up.add_argument("--nps", default="nps1", help="memory partition mode (node labeller label)")
    up.add_argument("--resource-strategy", default="single", choices=("single", "mixed"),
                    help="device plugin naming: amd.com/gpu, or amd.com/<partition>_<nps>")
    up.add_argument("--unhealthy", type=int, default=0, help="devices the device plugin reports unhealthy")
    up.add_argument("--no-portforward-tunnel", action="store_true",
                    help="no SPDY-over-WebSocket port-forward (an API server older than Kubernetes 1.30)")
    args = ap.parse_args(argv)
    c = LocalCluster(args.state, port=args.port, gpus=args.gpus, context=args.context, tls=args.tls,
                     gpu_partition=args.partition, memory_partition=args.nps, gpu_strategy=args.resource_strategy,
                     unhealthy_gpus=args.unhealthy, portforward_tunnel=not args.no_portforward_tunnel).start()
    c.api.reset_throttle(args.throttle_first, args.retry_after)
    c.kubelet.pull_seconds = args.pull_seconds
    kc = args.kubeconfig or os.path.join(args.state, "kubeconfig")
    c.write_kubeconfig(kc, args.namespace)
    print(f"ready server={c.server} kubeconfig={kc} docker=unix://{c.docker_sock} gpus={c.gpus}", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    c.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
