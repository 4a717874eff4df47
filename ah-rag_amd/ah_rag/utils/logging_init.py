"""Session event log (reference src/ah_rag/utils/logging_init.py:10-64): one JSON object per line
in <session_path>/events.jsonl, stamped with "ts". The reference prefers structlog when it is
installed and falls back to this plain writer; the on-disk format is the same."""
from __future__ import annotations

import json
import os
from datetime import datetime
from typing import Any


class JsonlLogger:
    def __init__(self, session_path: str, session_id: str, redact: bool = True) -> None:
        self.session_path = session_path
        self.session_id = session_id
        self.redact = redact
        os.makedirs(session_path, exist_ok=True)

    def info(self, **event: Any) -> None:
        if self.redact:
            for key in list(event):
                if key.lower() in {"api_key", "authorization"}:
                    event[key] = "[REDACTED]"
        event = {**event, "session_id": self.session_id, "ts": datetime.utcnow().isoformat() + "Z"}
        try:
            with open(os.path.join(self.session_path, "events.jsonl"), "a", encoding="utf-8") as f:
                f.write(json.dumps(event, ensure_ascii=False, default=str) + "\n")
        except Exception:
            pass


def get_logger(session_path: str, session_id: str, level: str = "normal", redact: bool = True) -> JsonlLogger:
    return JsonlLogger(session_path, session_id, redact=redact)
