"""Event-file framing (TFRecord + masked CRC32C) and metrics stream."""
import json
import struct

from distributed_char_rnn_amd.utils import tfevents
from distributed_char_rnn_amd.utils.metrics import MetricsLogger, progress_line


def test_crc32c_known_vector():
    assert tfevents.crc32c(b"123456789") == 0xE3069283


def test_event_file_roundtrip(tmp_path):
    w = tfevents.EventWriter(str(tmp_path))
    w.scalar("train_loss", 1.25, 3)
    w.histogram("logits", [0.0, 1.0, 2.0, 2.5], 3)
    w.close()
    recs = list(tfevents.read_records(w.path))
    assert len(recs) == 3
    assert b"brain.Event:2" in recs[0]
    assert b"train_loss" in recs[1] and struct.pack("<f", 1.25) in recs[1]
    assert b"logits" in recs[2]


def test_metrics_logger_and_progress_line(tmp_path):
    m = MetricsLogger(str(tmp_path))
    m.log({"step": 1, "loss": 2.0})
    m.scalar("train_loss", 2.0, 1)
    m.close()
    lines = (tmp_path / m.run_dir.split("/")[-1] / "metrics.jsonl").read_text().splitlines()
    assert json.loads(lines[0])["loss"] == 2.0
    s = progress_line(12, 100, 0, 3.14159, 0.05, 1000.0)
    assert s == "12/100 (epoch 0), train_loss = 3.142, time/batch = 0.050, chars/sec = 1000"
