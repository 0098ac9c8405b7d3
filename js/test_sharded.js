// One rank of glp_intopt sharded over processes (SURVEY.md §8(e)) through the
// JS boundary: gk_core.iosDriver with the communicator the environment
// describes (GK_WORLD_SIZE, GK_RANK, GK_COMM_ADDR; gk_core.comm).  For each
// MIP fixture named on the command line: the root LP (solve_lp's flow), then
// the sharded native search; prints one JSON line per fixture with the
// return code, status, objective and incumbent of this rank.
'use strict';
var fs = require('fs');
var path = require('path');
var U = require(path.join(__dirname, 'test_util.js'));
var core = U.core;

var dir = path.join(__dirname, '..', 'tests', 'golden');
process.argv.slice(2).forEach(function (name) {
    var fx = JSON.parse(fs.readFileSync(path.join(dir, 'mip_' + name + '.json'), 'utf8'));
    var mp = U.mipProblem(fx), lp = mp.lp;
    var T = {mip: lp, parm: U.iocp({msg_lev: 1})};
    if (!core.nativeIos(T)) throw new Error(name + ': not served natively');
    var ret = core.iosDriver(T, null);
    if (ret === 0) lp.mip_stat = (lp.mip_stat === 2) ? 5 : 4;   // solve_mip (glpapi09.js:82-92)
    var x = [];
    for (var j = 1; j <= lp.n; j++) x.push(lp.col[j].mipx);
    console.log(JSON.stringify({name: name, rank: parseInt(process.env.GK_RANK || '0', 10),
                                backend: core.comm() ? core.addon.commBackend(core.comm()) : 0, ret: ret,
                                mip_stat: lp.mip_stat, mip_obj: lp.mip_obj, x: x}));
});
