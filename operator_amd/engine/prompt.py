"""Prompt rendering for explanation requests.

The reference forwards ``AIProvider.spec.promptTemplate`` untouched to its
ai-interface service (J/service/AIInterfaceClient.java:82), which owns the
templating. Here the template is rendered on-node. Placeholders (``{name}``)
available to a custom template:

  podName, podNamespace, highestSeverity, significantEvents, totalEvents,
  events (the rendered top-k event block), analysis (AnalysisResult JSON)

Unknown placeholders are left verbatim; literal braces need no escaping
unless they form a ``{known}`` placeholder. Prompts are bounded by dropping
context lines / events (lowest-ranked first) until the token budget holds.
"""
from __future__ import annotations

import json
import re

from operator_amd.api.models import AnalysisResult

DEFAULT_TEMPLATE = (
    "You are Podmortem, a Kubernetes failure analyst. Given pattern-analysis results "
    "from a failed pod's logs, explain the most likely root cause and how to fix it. "
    "Answer with the sections \"Root Cause\", \"Evidence\" and \"Fix\".\n\n"
    "Pod {podNamespace}/{podName} failed. Highest severity: {highestSeverity}. "
    "Significant events: {significantEvents} of {totalEvents}.\n\n"
    "Matched failure patterns (most significant first):\n{events}\n\nAnalysis:\n"
)

_PH = re.compile(r"\{([A-Za-z_][A-Za-z0-9_]*)\}")


def render_events(result: AnalysisResult, top_k: int = 5, context: int | None = None) -> str:
    out = []
    for i, e in enumerate((result.events or [])[:top_k]):
        mp = e.matched_pattern
        head = (f"{i + 1}. [{mp.severity if mp else '?'}] {mp.name if mp else '?'} "
                f"(line {e.line_number}, score {e.score:.2f})")
        ctx = e.context or ([e.matched_line] if e.matched_line else [])
        if context is not None and ctx:
            mid = len(ctx) // 2
            ctx = ctx[max(0, mid - context): mid + context + 1]
        out.append(head + ("\n" + "\n".join("   | " + c[:240] for c in ctx) if ctx else ""))
    return "\n".join(out) if out else "(no known failure pattern matched)"


def render(result: AnalysisResult, template: str | None = None, top_k: int = 5, context: int | None = None) -> str:
    s = result.summary
    vals = {
        "podName": result.pod_name or "unknown",
        "podNamespace": result.pod_namespace or "default",
        "highestSeverity": (s.highest_severity if s else None) or "NONE",
        "significantEvents": str(s.significant_events if s else 0),
        "totalEvents": str(s.total_events if s else 0),
        "events": render_events(result, top_k, context),
    }
    tpl = template or DEFAULT_TEMPLATE

    def sub(m):
        k = m.group(1)
        if k == "analysis":
            return json.dumps(result.to_obj(), separators=(",", ":"))[:8000]
        return vals.get(k, m.group(0))

    return _PH.sub(sub, tpl)


# Shrink ladder: (events kept, context lines kept on each side of the match; None = all)
LADDER = ((5, None), (5, 2), (5, 1), (3, 0), (1, 0), (0, 0))


def render_bounded(result: AnalysisResult, tokenizer, max_tokens: int, template: str | None = None) -> list[int]:
    """Token ids of the rendered prompt, shrunk (context, then events) to fit ``max_tokens``."""
    return render_bounded_batch([(result, template)], tokenizer, max_tokens)[0]


def render_bounded_batch(items: list[tuple[AnalysisResult, str | None]], tokenizer, max_tokens: int) -> list[list[int]]:
    """``render_bounded`` for many prompts at once: every rung of the shrink ladder is
    ONE ``encode_batch`` call over the prompts still too long (the tokenizer's Rust
    core encodes them in parallel without the GIL), instead of one or more
    GIL-holding ``encode`` calls per prompt. Same result as the per-prompt loop."""
    out: list[list[int] | None] = [None] * len(items)
    todo = list(range(len(items)))
    last: dict[int, list[int]] = {}
    for top_k, ctx in LADDER:
        if not todo:
            break
        enc = tokenizer.encode_batch([render(items[i][0], items[i][1], top_k, ctx) for i in todo])
        nxt = []
        for i, ids in zip(todo, enc):
            if len(ids) <= max_tokens:
                out[i] = ids
            else:
                last[i] = ids
                nxt.append(i)
        todo = nxt
    for i in todo:
        out[i] = last[i][:max_tokens]
    return out  # type: ignore[return-value]
