/*
 * ref_cpu.c -- C port of the reference's enricher + advanced-metrics path.
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/ (mid-size parity checker) and by bench.py's
 * cpu_baseline leg (the timed CPU baseline).  Never linked into the product.
 *
 * "Go-shaped": it keeps the reference's per-flow cost structure -- IP addresses become
 * dotted strings (utils.Int2ip + net.IP.String, utils_linux.go:51-55), the cache is a
 * string-keyed map (cache.go:17-46,110-169), every metric builds its label values as
 * strings (types.go:418-505) and accumulates into a map keyed by the label tuple (what
 * GaugeVec.WithLabelValues does).  One thread runs enrich + every ProcessFlow per flow
 * (metrics_module.go:282-297); the reference pipelines those over two goroutines.
 *
 * Semantics restated from: enricher.go:102-183, types.go:109-368, forward.go:150-224,
 * drops.go:315-395, tcpflags.go:68-175, tcpretrans.go:247-298, dns.go:404-540,
 * flow_utils.go:33-305, metrics_module.go:205-264 -- identical to oracle/oracle.py,
 * which the reference's own tests pin (tests/test_oracle_kat.py).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- string map ---- */
typedef struct {
  char *key;
  void *val;
  uint64_t num;
} ent_t;
typedef struct {
  ent_t *e;
  size_t cap, n;
} smap_t;

static uint64_t shash(const char *s) {
  uint64_t h = 1469598103934665603ULL;
  for (; *s; ++s) h = (h ^ (unsigned char)*s) * 1099511628211ULL;
  return h;
}
static void smap_grow(smap_t *m);
static ent_t *smap_find(smap_t *m, const char *k, int create) {
  if (!m->cap) {
    if (!create) return NULL;
    m->cap = 1024;
    m->e = calloc(m->cap, sizeof(ent_t));
  }
  size_t i = shash(k) & (m->cap - 1);
  for (;;) {
    ent_t *e = &m->e[i];
    if (!e->key) {
      if (!create) return NULL;
      if (2 * (m->n + 1) > m->cap) {
        smap_grow(m);
        return smap_find(m, k, 1);
      }
      e->key = strdup(k);
      m->n++;
      return e;
    }
    if (!strcmp(e->key, k)) return e;
    i = (i + 1) & (m->cap - 1);
  }
}
static void smap_grow(smap_t *m) {
  smap_t o = *m;
  m->cap *= 2;
  m->n = 0;
  m->e = calloc(m->cap, sizeof(ent_t));
  for (size_t i = 0; i < o.cap; ++i)
    if (o.e[i].key) {
      ent_t *d = smap_find(m, o.e[i].key, 1);
      d->val = o.e[i].val;
      d->num = o.e[i].num;
      free(o.e[i].key);
    }
  free(o.e);
}
static void smap_free(smap_t *m, int free_vals) {
  for (size_t i = 0; i < m->cap; ++i)
    if (m->e[i].key) {
      free(m->e[i].key);
      if (free_vals) free(m->e[i].val);
    }
  free(m->e);
  memset(m, 0, sizeof *m);
}

/* ---------------------------------------------------------------- model ---------- */
enum { O_IP = 1, O_NS = 2, O_POD = 4, O_WL = 8, O_SVC = 16, O_PORT = 32 };
enum { F_FWD, F_DROP, F_TCPFLAGS, F_RETRANS, F_DNS };

typedef struct {
  char ns[128], pod[256], wk_kind[64], wk_name[256];
  int has_owner;
} endpoint_t;

typedef struct {
  uint32_t rcode, nresp;
  char *qtypes, *query, *ips;
} dns_t;

typedef struct {
  char name[128];
  char vec[64];
  int family, is_bytes, active, adv, has_src, has_dst, src_opts, dst_opts;
  int dns_kind; /* 1 request, 2 response */
  smap_t series; /* label tuple -> value */
} metric_t;

typedef struct {
  int remote;
  smap_t ip_to_ep; /* dotted ip -> endpoint* */
  endpoint_t **eps;
  size_t neps;
  dns_t *dns;
  size_t ndns, dns_cap;
  metric_t m[32];
  int nm;
  /* flattened output */
  char **out_metric, **out_labels;
  uint64_t *out_value;
  size_t nout;
} ref_t;

static const char *DROP_NAMES[7] = {"IPTABLE_RULE_DROP", "IPTABLE_NAT_DROP", "TCP_CONNECT_BASIC",
                                    "TCP_ACCEPT_BASIC", "TCP_CLOSE_BASIC", "CONNTRACK_ADD_DROP",
                                    "UNKNOWN_DROP"};
static const char *RCODES[6] = {"NOERROR", "FORMERR", "SERVFAIL", "NXDOMAIN", "NOTIMP", "REFUSED"};

static int parse_opts(const char **l, int n) {
  int o = 0;
  char b[64];
  for (int i = 0; i < n; ++i) {
    size_t k = 0;
    for (; l[i][k] && k < 63; ++k) b[k] = (char)((l[i][k] >= 'A' && l[i][k] <= 'Z') ? l[i][k] + 32 : l[i][k]);
    b[k] = 0;
    if (!strcmp(b, "ip")) o |= O_IP;
    else if (!strcmp(b, "namespace")) o |= O_NS;
    else if (!strcmp(b, "podname")) o |= O_POD;
    else if (!strcmp(b, "workload")) o |= O_WL;
    else if (!strcmp(b, "service")) o |= O_SVC;
    else if (!strcmp(b, "port")) o |= O_PORT;
  }
  return o;
}

static int contains_ci(const char *s, const char *sub) {
  char b[256];
  size_t k = 0;
  for (; s[k] && k < 255; ++k) b[k] = (char)((s[k] >= 'A' && s[k] <= 'Z') ? s[k] + 32 : s[k]);
  b[k] = 0;
  return strstr(b, sub) != NULL;
}

void *ref_create(int remote) {
  ref_t *r = calloc(1, sizeof(ref_t));
  r->remote = remote;
  return r;
}

/* Module.updateMetricsContexts (metrics_module.go:205-264). Returns 0, or -1 if the
 * reference would panic on the first matching flow. */
int ref_add_metric(void *h, const char *name, const char **src, int nsrc, int src_set,
                   const char **dst, int ndst, int dst_set) {
  ref_t *r = h;
  metric_t m;
  memset(&m, 0, sizeof m);
  snprintf(m.name, sizeof m.name, "%s", name);
  m.has_src = src_set;
  m.has_dst = r->remote ? dst_set : 0;
  m.src_opts = src_set ? parse_opts(src, nsrc) : 0;
  m.dst_opts = m.has_dst ? parse_opts(dst, ndst) : 0;
  m.adv = name[0] && (nsrc > 0 || ndst > 0);
  int make = 0;
  if (strstr(name, "forward")) {
    make = 1;
    m.family = F_FWD;
    m.active = !strcmp(name, "forward_count") || !strcmp(name, "forward_bytes");
    m.is_bytes = !strcmp(name, "forward_bytes");
    strcpy(m.vec, m.is_bytes ? "adv_forward_bytes" : "adv_forward_count");
  } else if (strstr(name, "drop")) {
    make = 1;
    m.family = F_DROP;
    m.active = !strcmp(name, "drop_count") || !strcmp(name, "drop_bytes");
    m.is_bytes = !strcmp(name, "drop_bytes");
    strcpy(m.vec, m.is_bytes ? "adv_drop_bytes" : "adv_drop_count");
  } else if (strstr(name, "tcp")) {
    if (contains_ci(name, "retrans")) {
      make = 1;
      m.family = F_RETRANS;
      m.active = 1;
      strcpy(m.vec, "adv_tcpretrans_count");
    } else if (contains_ci(name, "flag")) {
      make = 1;
      m.family = F_TCPFLAGS;
      m.active = 1;
      strcpy(m.vec, "adv_tcpflags_count");
    }
  } else if (strstr(name, "node_apiserver")) {
    make = 0;
  } else if (strstr(name, "dns") || strstr(name, "pktmon")) {
    if (contains_ci(name, "dns")) {
      make = 1;
      m.family = F_DNS;
      if (!strcmp(name, "dns_request_count")) m.dns_kind = 1;
      else if (!strcmp(name, "dns_response_count")) m.dns_kind = 2;
      else return -1;
      m.active = 1;
      strcpy(m.vec, m.dns_kind == 1 ? "adv_dns_request_count" : "adv_dns_response_count");
    }
  }
  if (!make) return 0;
  if (!r->remote && m.active && !m.has_src) return -1;
  for (int i = 0; i < r->nm; ++i)
    if (!strcmp(r->m[i].name, name)) {
      smap_free(&r->m[i].series, 0);
      r->m[i] = m;
      return 0;
    }
  if (r->nm >= 32) return -1;
  r->m[r->nm++] = m;
  return 0;
}

static void ip_str(uint32_t ip, char *b) {
  sprintf(b, "%u.%u.%u.%u", ip & 255u, (ip >> 8) & 255u, (ip >> 16) & 255u, ip >> 24);
}

/* Cache.UpdateRetinaEndpoint restated for IP ownership: later writers own an IP. */
int ref_add_endpoint(void *h, const char *ns, const char *pod, const char *wk_kind,
                     const char *wk_name, const uint32_t *ips, int nips) {
  ref_t *r = h;
  endpoint_t *e = calloc(1, sizeof *e);
  snprintf(e->ns, sizeof e->ns, "%s", ns);
  snprintf(e->pod, sizeof e->pod, "%s", pod);
  if (wk_kind) {
    e->has_owner = 1;
    snprintf(e->wk_kind, sizeof e->wk_kind, "%s", wk_kind);
    snprintf(e->wk_name, sizeof e->wk_name, "%s", wk_name ? wk_name : "");
  }
  r->eps = realloc(r->eps, (r->neps + 1) * sizeof(endpoint_t *));
  r->eps[r->neps++] = e;
  char b[20];
  for (int i = 0; i < nips; ++i) {
    ip_str(ips[i], b);
    smap_find(&r->ip_to_ep, b, 1)->val = e;
  }
  return 0;
}

int ref_add_dns(void *h, uint32_t rcode, const char *qtypes, const char *query, const char *ips,
                uint32_t nresp) {
  ref_t *r = h;
  if (r->ndns == r->dns_cap) {
    r->dns_cap = r->dns_cap ? 2 * r->dns_cap : 1024;
    r->dns = realloc(r->dns, r->dns_cap * sizeof(dns_t));
  }
  dns_t *d = &r->dns[r->ndns++];
  d->rcode = rcode;
  d->nresp = nresp;
  d->qtypes = strdup(qtypes);
  d->query = strdup(query);
  d->ips = strdup(ips);
  return (int)(r->ndns - 1);
}

/* ---------------------------------------------------------------- per flow ------- */
typedef struct {
  char sip[20], dip[20];
  uint32_t proto, verdict, tdir, reason, flags, dnstype, sport, dport, bytes, dns_id;
  endpoint_t *src, *dst;
} flow_t;

/* append getByDirectionValues (types.go:418-505) as "\x1f"-separated values */
static char *put(char *p, const char *s) {
  *p++ = '\x1f';
  size_t n = strlen(s);
  memcpy(p, s, n);
  return p + n;
}
static char *side_values(char *p, int opts, const flow_t *f, int dest) {
  const endpoint_t *ep = dest ? f->dst : f->src;
  char b[16];
  if (opts & O_IP) p = put(p, dest ? f->dip : f->sip);
  if (opts & O_NS) p = put(p, ep ? ep->ns : "unknown");
  if (opts & O_POD) p = put(p, ep ? ep->pod : "unknown");
  if (opts & O_WL) {
    if (ep && ep->has_owner) {
      p = put(p, ep->wk_kind);
      p = put(p, ep->wk_name);
    } else {
      p = put(p, "unknown");
      p = put(p, "unknown");
    }
  }
  if (opts & O_SVC) p = put(p, "unknown");
  if (opts & O_PORT) {
    if (f->proto == 6 || f->proto == 17) {
      sprintf(b, "%u", dest ? f->dport : f->sport);
      p = put(p, b);
    } else {
      p = put(p, "unknown");
    }
  }
  return p;
}
static void update(metric_t *m, const char *labels, uint64_t v) {
  ent_t *e = smap_find(&m->series, labels, 1);
  e->num += v;
}
static int is_api(const endpoint_t *e) {
  return e && !strcmp(e->ns, "kubernetes-apiserver") && !strcmp(e->pod, "kubernetes-apiserver");
}
static const char *tdir_name(uint32_t t, char *b) {
  if (t == 0) return "TRAFFIC_DIRECTION_UNKNOWN";
  if (t == 1) return "INGRESS";
  if (t == 2) return "EGRESS";
  sprintf(b, "%u", t);
  return b;
}
static const char *reason_name(uint32_t r, char *b) {
  if (r < 7) return DROP_NAMES[r];
  sprintf(b, "%u", r);
  return b;
}

static void process_metric(ref_t *r, metric_t *m, const flow_t *f) {
  char lab[4096], tb[16], rb[16];
  char *p;
  const int local = !r->remote;
  /* verdict / family filters */
  const char *flags[8];
  int nflags = 0;
  if (m->family == F_FWD && f->verdict != 1) return;
  if (m->family == F_DROP && f->verdict != 2) return;
  if (m->family == F_RETRANS && f->verdict != 15) return;
  if (m->family == F_TCPFLAGS) {
    if (f->verdict != 1 || f->proto != 6) return;
    uint32_t fl = f->flags; /* tcpflags.go:134-175 over AddTCPFlags bits */
    if (fl & 1) flags[nflags++] = "FIN";
    if ((fl & 2) && (fl & 16)) flags[nflags++] = "SYNACK";
    else {
      if (fl & 2) flags[nflags++] = "SYN";
      if (fl & 16) flags[nflags++] = "ACK";
    }
    if (fl & 4) flags[nflags++] = "RST";
    if (fl & 8) flags[nflags++] = "PSH";
    if (fl & 32) flags[nflags++] = "URG";
    if (!nflags) return;
  }
  char payload[3072];
  payload[0] = 0;
  if (m->family == F_DNS) {
    if (f->verdict != 16) return;
    if (f->dnstype == 0) return;
    if (m->dns_kind == 1 && f->dnstype != 1) return;
    if (m->dns_kind == 2 && f->dnstype != 2) return;
    const dns_t *d = &r->dns[f->dns_id];
    char *q = payload;
    char nb[16];
    if (f->dnstype == 1) {
      q = put(q, d->qtypes);
      q = put(q, d->query);
    } else {
      q = put(q, d->rcode < 6 ? RCODES[d->rcode] : "");
      q = put(q, d->qtypes);
      q = put(q, d->query);
      q = put(q, d->ips);
      sprintf(nb, "%u", d->nresp);
      q = put(q, nb);
    }
    *q = 0;
  }
  const uint64_t add = (m->is_bytes) ? f->bytes : 1;
  if (local) {
    /* getLocalCtxValues (types.go:379-416) */
    const int opts = m->src_opts;
    const int ing = f->dst && !is_api(f->dst) && opts;
    const int egr = f->src && !is_api(f->src) && opts;
    if (m->family == F_DNS) { /* dns.go:506-540 */
      int dest;
      if (ing && egr) dest = f->tdir == 1;
      else if (ing) dest = 1;
      else if (egr) dest = 0;
      else return;
      p = lab + sprintf(lab, "%s", payload);
      p = side_values(p, opts, f, dest);
      *p = 0;
      update(m, lab, 1);
      return;
    }
    for (int side = 0; side < 2; ++side) {
      const int dest = side == 0; /* ingress first, like processLocalCtxFlow */
      if (dest ? !ing : !egr) continue;
      const char *dir = dest ? "ingress" : "egress";
      if (m->family == F_TCPFLAGS) {
        for (int k = 0; k < nflags; ++k) {
          p = put(lab, flags[k]);
          p = side_values(p, opts, f, dest);
          *p = 0;
          update(m, lab, 1);
        }
        continue;
      }
      p = lab;
      if (m->family == F_DROP) p = put(p, reason_name(f->reason, rb));
      p = put(p, dir);
      p = side_values(p, opts, f, dest);
      *p = 0;
      update(m, lab, add);
    }
    return;
  }
  /* remote context: [prefix labels] + src values + dst values */
  char ctx[2048];
  char *c = ctx;
  const int with_ctx = m->family != F_FWD || m->adv;
  if (with_ctx && m->has_src) c = side_values(c, m->src_opts, f, 0);
  if (with_ctx && m->has_dst) c = side_values(c, m->dst_opts, f, 1);
  *c = 0;
  if (m->family == F_TCPFLAGS) {
    for (int k = 0; k < nflags; ++k) {
      p = put(lab, flags[k]);
      p += sprintf(p, "%s", ctx);
      update(m, lab, 1);
    }
    return;
  }
  p = lab;
  if (m->family == F_DNS) p += sprintf(p, "%s", payload);
  if (m->family == F_DROP) p = put(p, reason_name(f->reason, rb));
  if (m->family == F_FWD || m->family == F_DROP || m->family == F_RETRANS) p = put(p, tdir_name(f->tdir, tb));
  p += sprintf(p, "%s", ctx);
  update(m, lab, add);
}

int ref_process(void *h, const uint32_t *src, const uint32_t *dst, const uint32_t *bytes,
                const uint32_t *meta, const uint32_t *ports, const uint32_t *dns_id, size_t n) {
  ref_t *r = h;
  flow_t f;
  for (size_t i = 0; i < n; ++i) {
    /* producer -> flow (ToFlow, flow_utils.go:33-128) */
    ip_str(src[i], f.sip);
    ip_str(dst[i], f.dip);
    const uint32_t mt = meta[i];
    f.proto = mt & 0xFF;
    f.verdict = (mt >> 8) & 0xFF;
    if (f.verdict == 0) f.verdict = 1; /* ToFlow: 0 -> FORWARDED (flow_utils.go:94-96) */
    f.tdir = (mt >> 16) & 3;
    f.reason = (mt >> 18) & 7;
    f.flags = (f.verdict == 1 || f.verdict == 15) && f.proto == 6 ? (mt >> 21) & 0x3F : 0;
    f.dnstype = (mt >> 28) & 3;
    f.sport = ports ? ports[i] & 0xFFFF : 0;
    f.dport = ports ? ports[i] >> 16 : 0;
    f.bytes = bytes[i];
    f.dns_id = dns_id ? dns_id[i] : 0;
    if (f.verdict == 16 && f.dns_id >= r->ndns) return -1;
    /* enricher (enricher.go:102-135) */
    ent_t *e = smap_find(&r->ip_to_ep, f.sip, 0);
    f.src = e ? e->val : NULL;
    e = smap_find(&r->ip_to_ep, f.dip, 0);
    f.dst = e ? e->val : NULL;
    /* metrics module (metrics_module.go:282-297) */
    for (int k = 0; k < r->nm; ++k)
      if (r->m[k].active) process_metric(r, &r->m[k], &f);
  }
  return 0;
}

/* Flattens the series: labels are "\x1f"-separated values (label names are fixed per metric). */
size_t ref_finish(void *h) {
  ref_t *r = h;
  size_t n = 0;
  for (int k = 0; k < r->nm; ++k) n += r->m[k].series.n;
  r->out_metric = calloc(n + 1, sizeof(char *));
  r->out_labels = calloc(n + 1, sizeof(char *));
  r->out_value = calloc(n + 1, sizeof(uint64_t));
  size_t j = 0;
  for (int k = 0; k < r->nm; ++k) {
    smap_t *s = &r->m[k].series;
    for (size_t i = 0; i < s->cap; ++i)
      if (s->e[i].key) {
        r->out_metric[j] = r->m[k].vec;
        r->out_labels[j] = s->e[i].key;
        r->out_value[j] = s->e[i].num;
        ++j;
      }
  }
  r->nout = j;
  return j;
}

int ref_series(void *h, size_t i, const char **metric, const char **labels, uint64_t *value) {
  ref_t *r = h;
  if (i >= r->nout) return -1;
  *metric = r->out_metric[i];
  *labels = r->out_labels[i];
  *value = r->out_value[i];
  return 0;
}

void ref_destroy(void *h) {
  ref_t *r = h;
  if (!r) return;
  for (int k = 0; k < r->nm; ++k) smap_free(&r->m[k].series, 0);
  smap_free(&r->ip_to_ep, 0);
  for (size_t i = 0; i < r->neps; ++i) free(r->eps[i]);
  free(r->eps);
  for (size_t i = 0; i < r->ndns; ++i) {
    free(r->dns[i].qtypes);
    free(r->dns[i].query);
    free(r->dns[i].ips);
  }
  free(r->dns);
  free(r->out_metric);
  free(r->out_labels);
  free(r->out_value);
  free(r);
}
