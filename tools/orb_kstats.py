"""Prints the ORB kernels' mean durations from a rocprofv3 --stats directory: orb_kstats.py DIR TAG"""
import csv
import glob
import re
import sys

for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"orb_\w+", r["Name"])
        if m:
            print(sys.argv[2], m.group(0), round(float(r["AverageNs"]) / 1000, 1), "us")
