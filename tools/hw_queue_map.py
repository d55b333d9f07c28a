"""Which torch pool streams share a hardware queue (GPU_MAX_HW_QUEUES = 4 on
the box): a ~5 ms GEMM chain on stream A, then a tiny kernel on stream B;
B's kernel finishing before A's chain means separate queues, after it means
B queued behind A in one queue.  Streams are taken from torch's pool in
order (pool index = request order); the null stream is tested too.
    python tools/hw_queue_map.py [N]"""
import sys
import torch


def main():
  n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
  dev = torch.device("cuda")
  a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
  streams = [torch.cuda.Stream() for _ in range(n)]
  names = ["null"] + [f"pool{i}" for i in range(n)]
  objs = [torch.cuda.default_stream()] + streams
  x = torch.zeros(1, device=dev)

  def shares(sa, sb):
    torch.cuda.synchronize()
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0 = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(sa):
      e0.record()
      c = a
      for _ in range(40):
        c = c @ a
      ea.record()
    with torch.cuda.stream(sb):
      x.add_(1)
      eb.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(eb) > 0.5 * e0.elapsed_time(ea)

  rows = []
  for i, si in enumerate(objs):
    row = []
    for j, sj in enumerate(objs):
      row.append("." if i == j else ("X" if shares(si, sj) else " "))
    rows.append(row)
  print("A\\B      " + " ".join(f"{k:>2}" for k in range(len(objs))))
  for i, r in enumerate(rows):
    print(f"{names[i]:>7} {i:>2} " + " ".join(f"{c:>2}" for c in r), flush=True)


if __name__ == "__main__":
  main()
