"""Prints the top kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv, re, sys

def main(path, n=30):
  rows = list(csv.DictReader(open(path)))
  tot = sum(float(r["TotalDurationNs"]) for r in rows)
  for r in rows[:int(n)]:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Name"])[:90]
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} "
          f"{float(r['AverageNs'])/1e3:9.1f} us {100*float(r['TotalDurationNs'])/tot:5.1f}%  {name}")

if __name__ == "__main__":
  main(*sys.argv[1:])
