"""sparkmi counterpart of the reference's distributed_lstm.py: runs sparkmi.recipes.lstm
with one executor per spark.executor.instances (default: every visible MI355X; one CPU
executor without a GPU); any recipe flag overrides it, e.g. --world 8 --epochs 1."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sparkmi.recipes import lstm  # noqa: E402

if __name__ == "__main__":
    from sparkmi.api.session import Session
    conf = Session.builder.getOrCreate().sparkContext.getConf()
    executors_n = int(conf.get("spark.executor.instances", "0") or 0) or 1
    lstm.main(["--world", str(executors_n)] + sys.argv[1:])
