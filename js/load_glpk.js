// load_glpk.js — build the reference bundle with the MI355X shim and load it.
//
//   var glpk = require('./js/load_glpk.js')('/path/to/glpk.js');
//
// Same concatenation as the reference's build.sh:3
// (header + glpdebug.js + lib/*.js + footer) with js/gk_shim.js inserted
// before the footer.  The reference sources are read from refDir at run time;
// nothing of them is copied into this repository.
'use strict';
var fs = require('fs');
var os = require('os');
var path = require('path');

module.exports = function loadGlpk(refDir) {
    refDir = refDir || process.env.GLPK_REF || '/root/reference';
    var lib = path.join(refDir, 'lib');
    var files = fs.readdirSync(lib).filter(function (f) { return /\.js$/.test(f); }).sort();
    var parts = [fs.readFileSync(path.join(refDir, 'header'), 'utf8'),
                 fs.readFileSync(path.join(refDir, 'glpdebug.js'), 'utf8')];
    files.forEach(function (f) { parts.push(fs.readFileSync(path.join(lib, f), 'utf8')); });
    parts.push('var __gk_core_path = ' + JSON.stringify(path.join(__dirname, 'gk_core.js')) + ';');
    parts.push(fs.readFileSync(path.join(__dirname, 'gk_shim.js'), 'utf8'));
    parts.push(fs.readFileSync(path.join(refDir, 'footer'), 'utf8'));
    var dst = path.join(os.tmpdir(), 'glpk_mi355x_bundle_' + process.pid + '.js');
    fs.writeFileSync(dst, parts.join('\n'));
    return require(dst);
};
