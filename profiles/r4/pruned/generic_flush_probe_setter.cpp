// LDS-table flushes probe the home slots of all of a thread's keys at once
// (cb_flush); 0 = every key through gtab_insert (A/B)
static int g_flush_probe = 0;

int mr_agg_set_flush_probe(int on) {
  g_flush_probe = on ? 1 : 0;
  return 0;
}

