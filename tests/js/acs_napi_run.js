// TEST INFRASTRUCTURE: drive lib/acs_mi355x.node from Node the way a TS host would.
// usage: node acs_napi_run.js <dir>   (dir holds blob.bin, meta.json and the batch arrays
// written by tests/test_napi.py; results are written back into dir)
'use strict';
const fs = require('fs');
const path = require('path');
const addon = require(path.join(__dirname, '..', '..', 'access-control-srv_amd', 'lib', 'acs_mi355x.node'));

const dir = process.argv[2];
const rd = (f) => { const b = fs.readFileSync(path.join(dir, f)); return new Uint8Array(b.buffer, b.byteOffset, b.length); };
const meta = JSON.parse(fs.readFileSync(path.join(dir, 'meta.json'), 'utf8'));
const batch = { n: meta.n, rxCols: meta.rxCols, rxRows: meta.rxRows, candWords: meta.candWords,
                candWp: meta.candWp, candWr: meta.candWr, candRows: meta.candRows,
                candWsu: meta.candWsu, candWpu: meta.candWpu, candWv: meta.candWv };
for (const k of ['hdr', 'res', 'subj', 'act', 'roles', 'arena', 'rx', 'cand']) batch[k] = rd(k + '.bin');

(async () => {
  const h = addon.compile(rd('blob.bin'), 0);
  fs.writeFileSync(path.join(dir, 'out_sync.bin'), addon.isAllowed(h, batch));
  const outs = await Promise.all([addon.isAllowedAsync(h, batch), addon.isAllowedAsync(h, batch)]);
  fs.writeFileSync(path.join(dir, 'out_async.bin'), outs[1]);
  const w = addon.whatIsAllowed(h, batch);
  fs.writeFileSync(path.join(dir, 'wia_bits.bin'), Buffer.from(w.bits.buffer));
  fs.writeFileSync(path.join(dir, 'wia_obl_n.bin'), Buffer.from(w.oblN.buffer));
  fs.writeFileSync(path.join(dir, 'wia_out.bin'), w.out);
  // obligation-only pass over the first 16 requests, 3 set ranges, 128-entry logs
  const idx = new Uint32Array(16).map((_, i) => i);
  const o = addon.whatIsAllowedObl(h, batch, idx, 3, 128);
  fs.writeFileSync(path.join(dir, 'obl.bin'), Buffer.from(o.obl.buffer));
  fs.writeFileSync(path.join(dir, 'obl_n.bin'), Buffer.from(o.oblN.buffer));
  addon.free(h);
  console.log(JSON.stringify({ ok: true, words: w.bits.length / meta.n }));
})().catch((e) => { console.error(e); process.exit(1); });
