import sqlite3,glob,sys
db=glob.glob(sys.argv[1]+'/*.db')[0]
c=sqlite3.connect(db)
for r in c.execute("select substr(name,1,60), grid_x, count(*), round(avg(duration)/1000.0,1) from kernels where name like '%"+sys.argv[2]+"%' group by name, grid_x order by min(start)"):
    print(r)
