#!/usr/bin/env python3
"""configs[3]'s point set: the reference's own county centroids (data/county_centroids.csv,
3 233 rows: fips_code, name, longitude, latitude), as loaded by `load_centroids`
(src/sample_covid_data.rs:17-30), converted once to a data fixture.

The fixture holds only data — latitude / longitude in degrees as float64, in file order, and the
CSV's SHA-256 for provenance — so the configs[3] workload (workload.coords_workload) runs on the
reference's real centroid shape on the GPU box, where /root/reference does not exist. The
sampling itself (Zipf-weighted county draw + `uniform_in_square` jitter of side aug_len = 8 km,
src/sample_covid_data.rs:45-62, leader.rs:67-75, 331) happens in the workload generator.

Usage: python tests/golden/make_county_centroids.py [/root/reference/data/county_centroids.csv]
(writes tests/golden/county_centroids.npz)
"""
import csv
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data/county_centroids.csv"
    raw = open(src, "rb").read()
    text = raw.decode("utf-8-sig")   # the file starts with a byte-order mark
    rows = list(csv.DictReader(text.splitlines()))
    lat = np.array([float(r["latitude"]) for r in rows], np.float64)
    lon = np.array([float(r["longitude"]) for r in rows], np.float64)
    fips = np.array([int(r["fips_code"]) for r in rows], np.int32)
    out = os.path.join(HERE, "county_centroids.npz")
    np.savez_compressed(out, lat=lat, lon=lon, fips=fips, csv_sha256=np.array(hashlib.sha256(raw).hexdigest()))
    print(f"{out}: {lat.size} centroids, lat {lat.min():.2f}..{lat.max():.2f}, lon {lon.min():.2f}..{lon.max():.2f}")


if __name__ == "__main__":
    main()
