"""TEST INFRASTRUCTURE (checker only): a pure-Python restatement of Spark 2.1.0
MLUtils.parseLibSVMFile / parseLibSVMRecord (spark-mllib_2.11 2.1.0, pinned in the reference's
build.sbt:7-12; not vendored in the reference), used to check the native reader
fm_read_libsvm (fm_spark_amd/csrc/fm_libsvm.cpp).

  sc.textFile(path).map(_.trim).filter(line => !(line.isEmpty || line.startsWith("#")))
  items = line.split(' '); label = items.head.toDouble
  items.tail.filter(_.nonEmpty).map { item => val iv = item.split(':'); (iv(0).toInt - 1, iv(1).toDouble) }
  require(current > previous, "indices should be one-based and in ascending order ...")
  numFeatures = parsed.map { case (_, indices, _) => indices.lastOption.getOrElse(0) }.reduce(max) + 1
"""

import numpy as np


def parse_libsvm(text: str):
    labels, row_ptr, col, val = [], [0], [], []
    max_last = 0
    for raw in text.split("\n"):
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        items = line.split(" ")
        labels.append(float(items[0]))
        prev, last = -1, 0
        for it in items[1:]:
            if not it:
                continue
            iv = it.split(":")
            idx = int(iv[0]) - 1
            v = float(iv[1])
            if not idx > prev:
                raise ValueError(f"indices should be one-based and in ascending order; line {line!r}")
            prev = last = idx
            col.append(idx)
            val.append(v)
        max_last = max(max_last, last)
        row_ptr.append(len(col))
    return (np.asarray(labels, dtype=np.float64), np.asarray(row_ptr, dtype=np.int64),
            np.asarray(col, dtype=np.int32), np.asarray(val, dtype=np.float64), max_last + 1)
