"""Prometheus text exposition of oracle series (TEST INFRASTRUCTURE ONLY).

Restates what a scrape of Retina's AdvancedRegistry returns for the advanced metrics:
the vectors are created by exporter.CreatePrometheus{Gauge,Counter}VecForMetric
(pkg/exporter/prometheusexporter.go:46-66) with the names/Help strings of
forward.go:18-26,47-64, drops.go:18-23,42-60, tcpflags.go:18-24,43-51,
tcpretrans.go:18-24,43-51 (GaugeVec) and dns.go:21-30,50-66 (CounterVec), namespace
"networkobservability" (prometheusexporter.go:11).  The text layout is client_golang
v1.21.1's (go.mod:8; not in this image, so the layout rules below are restated from its
published text format 0.0.4, and pinned by the scrape the reference's docs print,
docs/06-Troubleshooting/basic-metrics.md:86-124 -> reference_kat.json exposition_sample): families
sorted by name, "# HELP" (backslash and newline escaped) and "# TYPE" lines, a metric's
label pairs sorted by label name, metrics of a family sorted by their label values,
label values escaped (backslash, double quote, newline), sample values formatted as
Go strconv.FormatFloat(v, 'g', -1, 64).
"""

from __future__ import annotations

from decimal import Decimal
from typing import Dict, Tuple

FAMILIES = {
    "networkobservability_adv_forward_count": ("gauge", "Total number of forwarded packets"),
    "networkobservability_adv_forward_bytes": ("gauge", "Total number of forwarded bytes"),
    "networkobservability_adv_drop_count": ("gauge", "Total number of dropped packets"),
    "networkobservability_adv_drop_bytes": ("gauge", "Total number of dropped bytes"),
    "networkobservability_adv_tcpflags_count": ("gauge", "Total number of packets by TCP flag"),
    "networkobservability_adv_tcpretrans_count": ("gauge", "Total number of TCP retransmitted packets"),
    "networkobservability_adv_dns_request_count": ("counter", "Total number of DNS query packets"),
    "networkobservability_adv_dns_response_count": ("counter", "Total number of DNS response packets"),
}


def go_format_float(v: float) -> str:
    """strconv.FormatFloat(v, 'g', -1, 64): shortest round-trip digits; %e form when the
    decimal exponent is < -4 or >= 6 (fmtG's precision for shortest digits), else %f."""
    if v == 0:
        return "0"
    sign = "-" if v < 0 else ""
    d = Decimal(repr(abs(float(v))))  # repr gives the shortest round-trip digits
    t = d.normalize().as_tuple()
    digits = "".join(map(str, t.digits))
    x = len(digits) - 1 + t.exponent  # decimal exponent of the first digit
    if x < -4 or x >= 6:
        m = digits[0] + ("." + digits[1:] if len(digits) > 1 else "")
        return "%s%se%s%02d" % (sign, m, "-" if x < 0 else "+", abs(x))
    if x >= 0:
        ip = digits[:x + 1].ljust(x + 1, "0")
        frac = digits[x + 1:]
        return sign + ip + ("." + frac if frac else "")
    return sign + "0." + "0" * (-x - 1) + digits


def _esc(s: str, quote: bool) -> str:
    s = s.replace("\\", "\\\\").replace("\n", "\\n")
    return s.replace('"', '\\"') if quote else s


def render(series: Dict[Tuple[str, Tuple[Tuple[str, str], ...]], int], families=None) -> str:
    """families: {name: (type, help)}, default the advanced metrics' FAMILIES (the basic
    registry's sample in tests/golden/reference_kat.json passes its own)."""
    families = FAMILIES if families is None else families
    fams: Dict[str, list] = {}
    for (metric, labels), v in series.items():
        fams.setdefault(metric, []).append((tuple(sorted(labels, key=lambda p: p[0])), v))
    out = []
    for metric in sorted(fams):
        typ, help_ = families[metric]
        out.append("# HELP %s %s\n# TYPE %s %s\n" % (metric, _esc(help_, False), metric, typ))
        for pairs, v in sorted(fams[metric], key=lambda e: [val for _, val in e[0]]):
            lab = ",".join('%s="%s"' % (k, _esc(val, True)) for k, val in pairs)
            out.append("%s%s %s\n" % (metric, "{%s}" % lab if pairs else "", go_format_float(float(v))))
    return "".join(out)
